"""GPU-resident PPO over the HIP env (d(ii), e): rollout collector + on-device rollout
buffer + GAE kernel (libquadswarm.so `qs_gae`) + minibatch update with one bucketed gradient all-reduce
per minibatch over RCCL.

Replaces what swarm_rl/sb_train.py:53-104 drives through stable_baselines3.PPO:
  * OnPolicyAlgorithm.collect_rollouts   -> PPOTrainer.collect_rollouts (no host round trip: obs, actions,
                                            rewards and dones stay in HBM; the env is the fused HIP step)
  * RolloutBuffer.compute_returns_and_advantage -> gae() (HIP kernel, time-major [T, I])
  * PPO.train                            -> PPOTrainer.train (same loss, clipping, advantage normalisation,
                                            grad-norm clip and Adam as SB3's defaults used by sb_train)
and the policy ActorCriticPolicyCustomSeparateWeights (swarm_rl/models/ActorCriticPolicyCustom.py:294-577)
with its QuadMultiEncoder (swarm_rl/models/quad_multi_model.py:250-353) -> SwarmActorCritic.

SB3 itself is not installed in this image: the PPO/GAE/squashed-Gaussian semantics are
restated from SB3's published algorithm and pinned by tests/test_ppo_cpu.py against the formulas
("parity unpinned" at the policy boundary).

Multi-GPU: one process per GPU, each rank steps its own env shard (drone_id_offset keys
the Philox streams), keeps its rollout/GAE/minibatches local, and after every minibatch backward the
gradients -- which autograd writes straight into ONE flat fp32 bucket -- are averaged with a single
all_reduce (RCCL over xGMI; gloo in the CPU tests).  Weights are broadcast from rank 0 at start.
"""
import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as NAT


# ----------------------------------------------------------------------------------------------
# policy (ActorCriticPolicyCustomSeparateWeights + QuadMultiEncoder)
# ----------------------------------------------------------------------------------------------
@dataclass
class PolicyConfig:
    """The model fields of swarm_rl/global_cfg.py the policy reads (defaults = global_cfg defaults;
    PolicyConfig.sb_train() = the parameter_sweep config of swarm_rl/sb_train.py:111-137)."""
    self_obs_dim: int = 7
    neighbor_obs_dim: int = 3
    num_use_neighbor_obs: int = 7
    obstacle_obs_dim: int = 0          # 9 (octomap SDF) when use_obstacles
    rnn_size: int = 256
    rnn_type: Optional[str] = None     # "full" -> ModelCoreMLP, else identity core
    rnn_num_layers: int = 2
    neighbor_hidden_size: int = 256
    neighbor_encoder_type: str = "attention"   # attention | mean_embed | mlp | no_encoder
    obst_hidden_size: int = 256
    nonlinearity: str = "tanh"
    policy_init_gain: float = 1.0
    decoder_mlp_layers: List[int] = field(default_factory=list)
    log_std_init: float = 0.0
    act_dim: int = 2

    @classmethod
    def for_env(cls, env_cfg, **over):
        """Dims from a QuadSwarmConfig (QuadMultiEncoder.__init__, quad_multi_model.py:254-275)."""
        so = NAT.SELF_OBS_DIM[NAT.OBS_REPR[env_cfg.obs_repr]]
        k = env_cfg.k_neighbors
        nd = NAT.NEIGHBOR_DIM[NAT.NEIGHBOR[env_cfg.neighbor_obs_type]] if k > 0 else 0
        kw = dict(self_obs_dim=so, neighbor_obs_dim=nd, num_use_neighbor_obs=k,
                  obstacle_obs_dim=9 if env_cfg.use_obstacles else 0, act_dim=env_cfg.act_dim)
        kw.update(over)
        return cls(**kw)

    @classmethod
    def sb_train(cls, env_cfg, **over):
        kw = dict(rnn_size=128, neighbor_hidden_size=128, rnn_type="full", rnn_num_layers=6,
                  neighbor_encoder_type="attention")
        kw.update(over)
        return cls.for_env(env_cfg, **kw)


def _act(cfg):
    # sample_factory.model.model_utils.nonlinearity
    return {"tanh": nn.Tanh, "relu": nn.ReLU, "elu": nn.ELU}[cfg.nonlinearity]()


def _mlp(cfg, sizes):
    layers = []
    for a, b in zip(sizes[:-1], sizes[1:]):
        layers += [nn.Linear(a, b), _act(cfg)]
    return nn.Sequential(*layers)


class NeighborMeanEmbed(nn.Module):
    """QuadNeighborhoodEncoderDeepsets (quad_multi_model.py:24-41): mean of per-neighbour embeddings."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        H = cfg.neighbor_hidden_size
        self.embedding_mlp = _mlp(cfg, [cfg.neighbor_obs_dim, H, H])

    def forward(self, self_obs, nbr):
        B, K = nbr.shape[0], self.cfg.num_use_neighbor_obs
        e = self.embedding_mlp(nbr.reshape(B * K, -1)).view(B, K, -1)
        return e.mean(dim=1)


class NeighborAttention(nn.Module):
    """QuadNeighborhoodEncoderAttention (quad_multi_model.py:44-101).

    Faithful to the reference's row pairing: neighbour rows are taken batch-major (row j = agent j // K,
    neighbour j % K) while the self-obs and mean-embedding copies are tiled batch-minor
    (`Tensor.repeat(K, 1)`, row j -> agent j % B), so row j pairs neighbour (j//K, j%K) with agent j % B's
    self obs.  That is what sb_train trains; reproducing it keeps checkpoints interchangeable."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        H = cfg.neighbor_hidden_size
        self.embedding_mlp = _mlp(cfg, [cfg.self_obs_dim + cfg.neighbor_obs_dim, H, H])
        self.neighbor_value_mlp = _mlp(cfg, [H, H, H])
        self.attention_mlp = nn.Sequential(nn.Linear(2 * H, H), _act(cfg), nn.Linear(H, H), _act(cfg),
                                           nn.Linear(H, 1))

    # split=True evaluates the two concatenating layers by their weight column blocks:
    #   cat(s.repeat(K,1), n) @ W^T + b   = n @ W_n^T + (s @ W_s^T + b)  broadcast over the K tiles
    #   cat(e, e_m.repeat(K,1)) @ A^T + a = e @ A_e^T + (e_m @ A_m^T + a) broadcast over the K tiles
    # (`Tensor.repeat(K, 1)` tiles batch-minor, so row j = (tile j // B, agent j % B) and the per-agent
    # term broadcasts over the leading K of a [K, B, H] view).  Same parameters and the same function;
    # the per-agent halves are computed once per agent instead of once per neighbour row, which removes
    # H*H of the 409 k MACs per neighbour row at H = 256 (and the two concatenated copies).  Rounding
    # differs from the concatenated GEMM only by summation order (tests/test_ppo_cpu.py pins it at fp64).
    split = True

    def forward(self, self_obs, nbr):
        B, K, H = nbr.shape[0], self.cfg.num_use_neighbor_obs, self.cfg.neighbor_hidden_size
        rows = nbr.reshape(B * K, -1)
        if not self.split:
            e = self.embedding_mlp(torch.cat((self_obs.repeat(K, 1), rows), dim=1))       # e_i
            h = self.neighbor_value_mlp(e)                                                # h_i
            e_mean = e.view(B, K, H).mean(dim=1)                                          # e_m
            score = self.attention_mlp(torch.cat((e, e_mean.repeat(K, 1)), dim=1)).view(B, K)
        else:
            so = self_obs.shape[1]
            l1, act = self.embedding_mlp[0], self.embedding_mlp[1]
            pre = F.linear(rows, l1.weight[:, so:]).view(K, B, H) + F.linear(self_obs, l1.weight[:, :so], l1.bias)
            e = self.embedding_mlp[2:](act(pre.view(B * K, H)))                           # e_i
            h = self.neighbor_value_mlp(e)                                                # h_i
            e_mean = e.view(B, K, H).mean(dim=1)                                          # e_m
            a1 = self.attention_mlp[0]
            pre = F.linear(e, a1.weight[:, :H]).view(K, B, H) + F.linear(e_mean, a1.weight[:, H:], a1.bias)
            score = self.attention_mlp[1:](pre.view(B * K, H)).view(B, K)
        w = torch.softmax(score, dim=1).view(B * K, 1)
        return (w * h).view(B, K, H).sum(dim=1)


class NeighborMlp(nn.Module):
    """QuadNeighborhoodEncoderMlp (quad_multi_model.py:104-122)."""

    def __init__(self, cfg):
        super().__init__()
        H = cfg.neighbor_hidden_size
        self.neighbor_mlp = _mlp(cfg, [cfg.neighbor_obs_dim * cfg.num_use_neighbor_obs, H, H, H])

    def forward(self, self_obs, nbr):
        return self.neighbor_mlp(nbr.reshape(nbr.shape[0], -1))


class QuadMultiEncoder(nn.Module):
    """quad_multi_model.py:250-353: self encoder (2 x Linear+act of rnn_size), optional neighbour
    encoder, optional obstacle encoder, then feed_forward Linear -> 2*rnn_size + Tanh."""

    def __init__(self, cfg: PolicyConfig):
        super().__init__()
        self.cfg = cfg
        R = cfg.rnn_size
        self.self_encoder = _mlp(cfg, [cfg.self_obs_dim, R, R])
        self.all_neighbor_obs_size = cfg.neighbor_obs_dim * cfg.num_use_neighbor_obs
        self.neighbor_encoder = None
        if cfg.num_use_neighbor_obs > 0:
            t = cfg.neighbor_encoder_type
            if t == "attention":
                self.neighbor_encoder = NeighborAttention(cfg)
            elif t == "mean_embed":
                self.neighbor_encoder = NeighborMeanEmbed(cfg)
            elif t == "mlp":
                self.neighbor_encoder = NeighborMlp(cfg)
            elif t != "no_encoder":
                raise NotImplementedError(t)
        out = R + (cfg.neighbor_hidden_size if self.neighbor_encoder is not None else 0)
        self.obstacle_encoder = None
        if cfg.obstacle_obs_dim:
            O = cfg.obst_hidden_size
            self.obstacle_encoder = _mlp(cfg, [cfg.obstacle_obs_dim, O, O])
            out += O
        self.feed_forward = nn.Sequential(nn.Linear(out, 2 * R), nn.Tanh())
        self.out_size = 2 * R

    def forward(self, obs, nbr_out=None, l0=None, ff=None):
        """nbr_out: the neighbour encoder's output computed elsewhere (the fused update, encoder_train.py); l0(lin,
        obs): the self encoder's first Linear evaluated elsewhere (FusedAttentionTrain.self_layer0); ff(lin, x): the
        feed_forward's Linear + Tanh evaluated elsewhere (FusedAttentionTrain.feed_forward), x a tensor or, for the
        feed_forward, the list of parts to concatenate."""
        so, na = self.cfg.self_obs_dim, self.all_neighbor_obs_size
        self_obs = obs[:, :so]
        se = self.self_encoder
        if l0 is not None and len(se) > 1:
            s1 = se[1](l0(se[0], obs))
            if ff is not None and len(se) == 4 and isinstance(se[2], nn.Linear) and isinstance(se[3], nn.Tanh):
                parts = [ff(se[2], s1)]   # the second Linear + Tanh (tanh inputs) evaluated elsewhere
            else:
                parts = [se[2:](s1)]
        else:
            parts = [se(self_obs)]
        if nbr_out is not None:
            parts.append(nbr_out)
        elif self.neighbor_encoder is not None:
            nbr = obs[:, so:so + na].reshape(obs.shape[0], self.cfg.num_use_neighbor_obs, -1)
            parts.append(self.neighbor_encoder(self_obs, nbr))
        if self.obstacle_encoder is not None:
            parts.append(self.obstacle_encoder(obs[:, so + na:]))
        if ff is not None and isinstance(self.feed_forward[0], nn.Linear):
            return ff(self.feed_forward[0], parts)   # the hook concatenates (or reads the parts in place)
        x = torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]
        return self.feed_forward(x)


class SwarmActorCritic(nn.Module):
    """ActorCriticPolicyCustomSeparateWeights (ActorCriticPolicyCustom.py:294-577): separate actor and
    critic towers (encoder -> ModelCoreMLP [rnn_type 'full'] or identity -> MlpDecoder), action_net +
    state-independent log_std feeding SB3's SquashedDiagGaussianDistribution, value_net.

    Initialisation as the reference: initialize_weights only touches modules whose type *is* nn.Linear
    (`:392-396`), so of the listed modules only action_net and value_net get xavier_uniform(gain); the
    encoders/cores keep PyTorch's default Linear init."""

    def __init__(self, cfg: PolicyConfig):
        super().__init__()
        self.cfg = cfg
        self.actor_encoder = QuadMultiEncoder(cfg)
        self.critic_encoder = QuadMultiEncoder(cfg)
        full = cfg.rnn_type == "full" and cfg.rnn_num_layers > 0
        enc = self.actor_encoder.out_size
        core_sizes = [enc] + [cfg.rnn_size] * cfg.rnn_num_layers
        self.actor_core = _mlp(cfg, core_sizes) if full else nn.Sequential()
        self.critic_core = _mlp(cfg, core_sizes) if full else nn.Sequential()
        lat = cfg.rnn_size if full else enc
        self.actor_decoder = _mlp(cfg, [lat] + list(cfg.decoder_mlp_layers))
        self.critic_decoder = _mlp(cfg, [lat] + list(cfg.decoder_mlp_layers))
        dec = cfg.decoder_mlp_layers[-1] if cfg.decoder_mlp_layers else lat
        self.action_net = nn.Linear(dec, cfg.act_dim)
        self.log_std = nn.Parameter(torch.ones(cfg.act_dim) * cfg.log_std_init)
        self.value_net = nn.Linear(dec, 1)
        for m in (self.value_net, self.action_net):
            nn.init.xavier_uniform_(m.weight.data, gain=cfg.policy_init_gain)

    # ---- towers ----
    def actor_latent(self, obs):
        return self.actor_decoder(self.actor_core(self.actor_encoder(obs)))

    def predict_values(self, obs):
        return self.value_net(self.critic_decoder(self.critic_core(self.critic_encoder(obs))))

    # ---- SB3 API ----
    def forward(self, obs, deterministic=False):
        """(actions in [-1,1], values [B,1], log_prob [B]) -- ActorCriticPolicyCustom.py:515-536."""
        mean = self.action_net(self.actor_latent(obs))
        values = self.predict_values(obs)
        if deterministic:
            actions = torch.tanh(mean)
        else:
            actions = torch.tanh(mean + torch.randn_like(mean) * self.log_std.exp())
        return actions, values, squashed_log_prob(mean, self.log_std, actions)

    def evaluate_actions(self, obs, actions, nbr=None, l0=None, ff=None):
        """(values, log_prob, entropy=None) -- ActorCriticPolicyCustom.py:538-566.  nbr: (actor, critic) neighbour
        encoder outputs from the fused update (encoder_train.FusedAttentionTrain), else the torch encoders run;
        l0 / ff: the fused update's self-encoder first layer and feed_forward (FusedAttentionTrain.self_layer0 /
        .feed_forward), with nbr only."""
        if nbr is None:
            mean = self.action_net(self.actor_latent(obs))
            return self.predict_values(obs), squashed_log_prob(mean, self.log_std, actions), None
        mean = head_linear(self.action_net,
                           self.actor_decoder(self.actor_core(self.actor_encoder(obs, nbr[0], l0, ff))))
        values = head_linear(self.value_net,
                             self.critic_decoder(self.critic_core(self.critic_encoder(obs, nbr[1], l0, ff))))
        return values, squashed_log_prob(mean, self.log_std, actions), None

    def predict(self, obs, deterministic=True):
        return torch.tanh(self.action_net(self.actor_latent(obs))) if deterministic else self.forward(obs)[0]

    # ---- checkpoints interchangeable with the reference's policy ----
    # The reference's module tree differs only in two wrapper levels: ModelCoreMLP keeps its layers in `.core`
    # (ActorCriticPolicyCustom.py:260-276) and MlpDecoder in `.mlp` (sample_factory); every other parameter
    # name (encoders, attention MLPs, feed_forward, action_net, log_std, value_net) is the same.
    _REF_WRAP = (("actor_core.", "actor_core.core."), ("critic_core.", "critic_core.core."),
                 ("actor_decoder.", "actor_decoder.mlp."), ("critic_decoder.", "critic_decoder.mlp."))

    @classmethod
    def reference_key(cls, key):
        """This module's parameter name -> ActorCriticPolicyCustomSeparateWeights' name for it."""
        for ours, ref in cls._REF_WRAP:
            if key.startswith(ours):
                return ref + key[len(ours):]
        return key

    @classmethod
    def from_reference_key(cls, key):
        for ours, ref in cls._REF_WRAP:
            if key.startswith(ref):
                return ours + key[len(ref):]
        return key

    def reference_state_dict(self):
        """state_dict under the reference policy's names (loadable by ActorCriticPolicyCustomSeparateWeights)."""
        return {self.reference_key(k): v for k, v in self.state_dict().items()}

    def load_reference_state_dict(self, sd, strict=True):
        """Load a state_dict of the reference's ActorCriticPolicyCustomSeparateWeights (e.g. the `policy` entry
        of an SB3 checkpoint of sb_train) -- same architecture, same function."""
        return self.load_state_dict({self.from_reference_key(k): v for k, v in sd.items()}, strict=strict)


_LOG_SQRT_2PI = 0.5 * math.log(2 * math.pi)


class _HeadLinearFn(torch.autograd.Function):
    """A head Linear (action_net / value_net: [B, d] -> [B, n], n <= 8) whose weight gradient g^T x is formed as a
    split-K batched product over row chunks and summed: the library's one skinny [n x B] x [B x d] GEMM runs at
    ~2 TF/s at the update's 262 144 rows.  Same function, fp32 (the chunk sums reassociate the row sum)."""

    CHUNK = 4096

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        B, d = x.shape
        c = _HeadLinearFn.CHUNK
        nb = B // c
        gw = torch.bmm(g[:nb * c].reshape(nb, c, -1).transpose(1, 2), x[:nb * c].reshape(nb, c, d)).sum(0)
        if nb * c < B:
            gw = gw + g[nb * c:].t().mm(x[nb * c:])
        gx = g.mm(weight) if ctx.needs_input_grad[0] else None
        return gx, gw, g.sum(0)


def head_linear(lin, x):
    """lin(x), with the split-K weight gradient for a large batch (_HeadLinearFn)."""
    if x.shape[0] >= 8 * _HeadLinearFn.CHUNK and lin.out_features <= 8 and torch.is_grad_enabled():
        return _HeadLinearFn.apply(x, lin.weight, lin.bias)
    return lin(x)


def squashed_log_prob(mean, log_std, actions, epsilon=1e-6):
    """SB3 SquashedDiagGaussianDistribution.log_prob(actions) with gaussian_actions recovered by
    TanhBijector.inverse (atanh of the action clamped to +-(1 - float32 eps)), minus the tanh Jacobian
    sum(log(1 - a^2 + 1e-6))."""
    eps = torch.finfo(actions.dtype).eps
    y = actions.clamp(-1.0 + eps, 1.0 - eps)
    g = 0.5 * (y.log1p() - (-y).log1p())
    z = (g - mean) * torch.exp(-log_std)
    lp = (-0.5 * z * z - log_std - _LOG_SQRT_2PI).sum(dim=1)
    return lp - torch.log(1 - actions * actions + epsilon).sum(dim=1)


# ----------------------------------------------------------------------------------------------
# GAE (HIP kernel behind the C ABI)
# ----------------------------------------------------------------------------------------------
def gae(rewards, values, episode_starts, last_values, last_dones, gamma=0.99, gae_lambda=0.95,
        advantages=None, returns=None):
    """RolloutBuffer.compute_returns_and_advantage on device via qs_gae.  rewards/values [T, I] fp32,
    episode_starts [T, I] u8, last_values [I] fp32, last_dones [I] u8 (all CUDA, contiguous).
    Returns (advantages, returns) [T, I].  No CPU path: a non-CUDA tensor is an error."""
    T, I = rewards.shape
    ts = (rewards, values, episode_starts, last_values, last_dones)
    if not all(t.is_cuda and t.is_contiguous() for t in ts):
        raise NAT.QuadSwarmError("gae(): all inputs must be contiguous HIP device tensors")
    if rewards.dtype != torch.float32 or values.dtype != torch.float32 or last_values.dtype != torch.float32 \
            or episode_starts.dtype != torch.uint8 or last_dones.dtype != torch.uint8:
        raise NAT.QuadSwarmError("gae(): rewards/values/last_values fp32, episode_starts/last_dones uint8")
    if values.shape != (T, I) or episode_starts.shape != (T, I) or last_values.numel() != I \
            or last_dones.numel() != I:
        raise NAT.QuadSwarmError("gae(): shape mismatch")
    if advantages is None:
        advantages = torch.empty_like(rewards)
    if returns is None:
        returns = torch.empty_like(rewards)
    s = torch.cuda.current_stream(rewards.device).cuda_stream
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    NAT.check(NAT.lib().qs_gae(p(rewards), p(values), p(episode_starts), p(last_values), p(last_dones),
                               p(advantages), p(returns), T, I, float(gamma), float(gae_lambda),
                               ctypes.c_void_p(s)), "qs_gae")
    return advantages, returns


# ----------------------------------------------------------------------------------------------
# GEMM solution table
# ----------------------------------------------------------------------------------------------
GEMM_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "tunableop_gfx950.csv")


def use_gemm_table(path=GEMM_TABLE):
    """Pin the policy's fp32 GEMMs to the hipBLASLt/rocBLAS solutions measured fastest on MI355X for the
    bench shapes (PyTorch TunableOp in read-only mode; tools/gpu_check.sh `tune*` regenerates the table).
    Shapes not in the table keep the library default.  Returns True when the table was loaded."""
    if not (torch.cuda.is_available() and os.path.exists(path)):
        return False
    if "gfx950" not in torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName:
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    return bool(tun.read_file(path))


# ----------------------------------------------------------------------------------------------
# trainer
# ----------------------------------------------------------------------------------------------
@dataclass
class PPOConfig:
    """SB3 PPO as constructed by sb_train.py:53-65 (global_cfg.py:21-29) + SB3 defaults."""
    n_steps: int = 512
    batch_size: int = 1024
    n_epochs: int = 10
    gamma: float = 0.99
    gae_lambda: float = 0.95
    learning_rate: float = 1e-4
    clip_range: float = 0.2
    ent_coef: float = 0.0
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    normalize_advantage: bool = True
    adam_eps: float = 1e-8      # the reference rebuilds Adam with torch defaults (ActorCriticPolicyCustom.py:348)


class FlatGradBucket:
    """All parameter .grad tensors as views of one flat fp32 buffer: autograd accumulates in place into
    it, so the data-parallel average is ONE all_reduce per minibatch (the DDP single-bucket case; the
    sb_train policy is ~0.6 M params = 2.4 MB) and grad-norm clipping is one norm over the bucket."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero(self):
        self.flat.zero_()

    def check_bound(self):
        base, end = self.flat.data_ptr(), self.flat.data_ptr() + 4 * self.flat.numel()
        return all(p.grad is not None and base <= p.grad.data_ptr() < end for p in self.params)

    def all_reduce_mean(self, group=None):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.flat, group=group)
            self.flat.div_(dist.get_world_size(group))

    def clip_norm_(self, max_norm):
        """torch.nn.utils.clip_grad_norm_ semantics over the bucket; returns the pre-clip norm (tensor)."""
        norm = torch.linalg.vector_norm(self.flat, dtype=torch.float64).float()   # fp64 accumulation
        self.flat.mul_(torch.clamp(max_norm / (norm + 1e-6), max=1.0))
        return norm


class RolloutStorage:
    """SB3 RolloutBuffer, HBM-resident and time-major: [T, I, ...] so a time slice is contiguous for the
    collector and the GAE kernel reads every time step as one coalesced row."""

    def __init__(self, T, I, obs_dim, act_dim, device):
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
        self.T, self.I = T, I
        self.obs = z(T, I, obs_dim)
        self.actions = z(T, I, act_dim)
        self.rewards = z(T, I)
        self.values = z(T, I)
        self.log_probs = z(T, I)
        self.episode_starts = z(T, I, dt=torch.uint8)
        self.advantages = z(T, I)
        self.returns = z(T, I)

    def flat(self, name):
        t = getattr(self, name)
        return t.view(self.T * self.I, *t.shape[2:])


class PPOTrainer:
    """OnPolicyAlgorithm.collect_rollouts + PPO.train over a device env.

    env: QuadSwarmEnv (or any object with .I, .obs_dim, .act_dim, .reset() -> obs [I, od] and
    .step(actions) -> (obs, rew, done, term) returning device tensors).  gae_fn is for tests that run
    the trainer on a CPU stand-in env; the default is the HIP kernel."""

    def __init__(self, env, policy: SwarmActorCritic, cfg: PPOConfig = None, device=None, seed=0,
                 gae_fn=None, group=None, fused_rollout=True, rollout_precision="fp32", update_precision="fp32"):
        import torch.distributed as dist

        self.env, self.policy, self.cfg = env, policy, cfg or PPOConfig()
        self.device = torch.device(device) if device is not None else next(policy.parameters()).device
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        # data parallel: rank r steps its own env shard; num_timesteps counts every rank's agents (the reference's
        # one VecEnv over all envs), so total_timesteps / save_freq / eval_freq keep their global meaning
        self.world_size = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        if self.distributed:
            for p in policy.parameters():   # identical weights on every rank
                dist.broadcast(p.data, src=0, group=group)
        self.bucket = FlatGradBucket(policy.parameters())
        self.optimizer = torch.optim.Adam(self.bucket.params, lr=self.cfg.learning_rate, eps=self.cfg.adam_eps)
        self.storage = RolloutStorage(self.cfg.n_steps, env.I, env.obs_dim, env.act_dim, self.device)
        self.gae_fn = gae_fn or gae
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.num_timesteps = 0
        self.env_steps = 0          # VecEnv steps taken (SubprocVecEnvCustom.batch)
        self.iterations = 0
        self.callbacks = []
        self.last_obs = None
        self.last_done = torch.zeros(env.I, dtype=torch.uint8, device=self.device)
        self.last_values = torch.zeros(env.I, dtype=torch.float32, device=self.device)
        # the rollout's policy evaluations through the fused HIP attention encoders (policy_fused.py) where
        # the policy has that encoder; the update keeps the torch module (autograd)
        self.fused = None
        if fused_rollout and self.device.type == "cuda":
            from .policy_fused import FusedRolloutPolicy, supports
            if supports(policy):
                self.fused = FusedRolloutPolicy(policy, precision=rollout_precision)
        # the update's neighbour encoders: torch autograd ("fp32") or the fused split-f16 kernels ("x3",
        # encoder_train.py: forward + backward on the matrix cores, fp32-equivalent products)
        if update_precision not in ("fp32", "x3"):
            raise ValueError("update_precision must be 'fp32' or 'x3'")
        self.update_precision = update_precision
        self.fused_update = None
        if update_precision == "x3":
            if self.device.type != "cuda":
                raise NAT.QuadSwarmError("update_precision='x3' needs a HIP device")
            from .encoder_train import FusedAttentionTrain
            self.fused_update = FusedAttentionTrain(policy)

    def reset(self):
        self.last_obs = self.env.reset()
        self.last_done.fill_(1)      # SB3: _last_episode_starts = ones after reset

    @torch.no_grad()
    def collect_rollouts(self, callbacks=()):
        """OnPolicyAlgorithm.collect_rollouts: n_steps env steps into the rollout buffer, then GAE.  After every env
        step each callback's on_step(StepContext) runs (SB3 order: num_timesteps already advanced); one returning
        False stops the rollout and the method returns False (no GAE), like SB3."""
        if self.last_obs is None:
            self.reset()
        st, pol = self.storage, self.policy
        pol.train(False)
        fwd = pol
        if self.fused is not None:
            self.fused.refresh()      # the weights the last update left
            fwd = self.fused
        from .callbacks import StepContext
        for cb in callbacks:
            cb.on_rollout_start(self)
        for t in range(self.cfg.n_steps):
            st.obs[t].copy_(self.last_obs)
            actions, values, logp = fwd(st.obs[t])
            st.actions[t].copy_(actions)
            st.values[t].copy_(values.view(-1))
            st.log_probs[t].copy_(logp)
            st.episode_starts[t].copy_(self.last_done)
            obs, rew, done, _ = self.env.step(st.actions[t])   # squashed actions are inside the box
            st.rewards[t].copy_(rew)
            self.last_done.copy_(done)
            self.last_obs = obs
            self.num_timesteps += self.env.I * self.world_size
            self.env_steps += 1
            if callbacks:
                ctx = StepContext(self, t, obs, rew, done, st.actions[t])
                go = True
                for cb in callbacks:
                    go = cb.on_step(ctx) is not False and go
                if not go:
                    return False
        self.last_values.copy_(fwd.predict_values(self.last_obs).view(-1))
        if self.fused is not None:
            self.fused.check_inputs()   # x3: the rollout's observations stayed inside the split-f16 range
        self.gae_fn(st.rewards, st.values, st.episode_starts, self.last_values, self.last_done,
                    self.cfg.gamma, self.cfg.gae_lambda, st.advantages, st.returns)
        for cb in callbacks:
            cb.on_rollout_end(self)
        return True

    def train(self, max_updates=None):
        """PPO.train: n_epochs over shuffled minibatches of the flattened rollout (max_updates cuts the
        pass short -- warm-up only)."""
        c, st, pol = self.cfg, self.storage, self.policy
        pol.train(True)
        n = st.T * st.I
        obs, act, old_lp = st.flat("obs"), st.flat("actions"), st.flat("log_probs")
        adv_all, ret_all, old_v = st.flat("advantages"), st.flat("returns"), st.flat("values")
        acc = torch.zeros(6, dtype=torch.float64, device=self.device)
        n_mb = 0
        # the fused x3 encoders only where the rollout's observations are inside their split-f16 range (one check per
        # update, whatever the rollout's precision); a weight out of range falls back per minibatch (encodings -> None)
        fused = self.fused_update if self.fused_update is not None and self.fused_update.obs_in_range(obs) else None
        for _ in range(c.n_epochs):
            perm = torch.randperm(n, device=self.device, generator=self.gen)
            for s in range(0, n, c.batch_size):
                idx = perm[s:s + c.batch_size]
                ob = obs[idx]
                nbr = fused.encodings(ob) if fused is not None else None
                values, logp, entropy = pol.evaluate_actions(ob, act[idx], nbr=nbr,
                                                             l0=fused.self_layer0 if nbr is not None else None,
                                                             ff=fused.feed_forward if nbr is not None else None)
                values = values.flatten()
                adv = adv_all[idx]
                if c.normalize_advantage and idx.numel() > 1:
                    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
                ratio = torch.exp(logp - old_lp[idx])
                pl1 = adv * ratio
                pl2 = adv * torch.clamp(ratio, 1 - c.clip_range, 1 + c.clip_range)
                policy_loss = -torch.min(pl1, pl2).mean()
                value_loss = F.mse_loss(ret_all[idx], values)
                entropy_loss = -torch.mean(-logp) if entropy is None else -torch.mean(entropy)
                loss = policy_loss + c.ent_coef * entropy_loss + c.vf_coef * value_loss
                self.bucket.zero()
                loss.backward()
                self.bucket.all_reduce_mean(self.group)
                self.bucket.clip_norm_(c.max_grad_norm)
                self.optimizer.step()
                with torch.no_grad():
                    lr = logp - old_lp[idx]
                    acc += torch.stack([policy_loss.detach(), value_loss.detach(), entropy_loss.detach(),
                                        ((ratio - 1).abs() > c.clip_range).float().mean(),
                                        torch.mean((torch.exp(lr) - 1) - lr), loss.detach()]).double()
                n_mb += 1
                if max_updates is not None and n_mb >= max_updates:
                    break
            if max_updates is not None and n_mb >= max_updates:
                break
        a = (acc / max(n_mb, 1)).tolist()
        yv, yt = old_v, ret_all
        ev = 1.0 - float(torch.var(yt - yv) / torch.var(yt)) if float(torch.var(yt)) > 0 else float("nan")
        return dict(policy_gradient_loss=a[0], value_loss=a[1], entropy_loss=a[2], clip_fraction=a[3],
                    approx_kl=a[4], loss=a[5], explained_variance=ev, n_updates=n_mb)

    def learn_iteration(self):
        self.collect_rollouts()
        stats = self.train()
        self.iterations += 1
        return stats

    def learn(self, total_timesteps, callback=None):
        """OnPolicyAlgorithm.learn as sb_train calls it (sb_train.py:93-98): rollouts + updates until
        num_timesteps reaches total_timesteps, with the callbacks' hooks (quadswarm_amd.callbacks).  Returns the
        last update's stats."""
        cbs = [] if callback is None else (list(callback) if isinstance(callback, (list, tuple)) else [callback])
        self.callbacks = cbs
        for cb in cbs:
            cb.on_training_start(self)
        stats = {}
        while self.num_timesteps < total_timesteps:
            if not self.collect_rollouts(cbs):
                break
            stats = self.train()
            self.iterations += 1
            for cb in cbs:
                cb.on_iteration_end(self)
        for cb in cbs:
            cb.on_training_end(self)
        return stats

    # ---- checkpoint / resume (sb_train: CheckpointCallback + model.save, sb_train.py:99-106) ----
    CKPT_FORMAT = "quadswarm_amd.PPOTrainer/2"
    ENV_PARAMS = ("seed", "ep_len", "rew_pos", "rew_effort", "rew_crash", "rew_orient", "rew_spin", "quadcol_bin",
                  "quadcol_bin_smooth_max", "quadcol_bin_obst")

    def _shard_state(self):
        """This rank's part of a checkpoint: its env snapshot (qs_get_state: drone and env state incl. the per-env
        Philox counters, capture radii, pillar maps) and runtime env parameters, the current observation / episode
        starts / bootstrap values, the replay wrapper's device state, and its random generators."""
        env = self.env
        u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).clone()  # noqa: E731
        sh = {"rank": self.rank,
              "gen": self.gen.get_state(), "device_rng": torch.cuda.get_rng_state(self.device)
              if self.device.type == "cuda" else torch.get_rng_state(),
              "last_obs": None if self.last_obs is None else self.last_obs.detach().cpu().clone(),
              "last_done": self.last_done.cpu().clone(), "last_values": self.last_values.cpu().clone()}
        if hasattr(env, "get_state"):
            sh["env_state"] = u8(env.get_state())
            # the runtime parameters qs_set_param may have changed (seed, reward annealing, episode length)
            sh["env_params"] = {}
            for k in self.ENV_PARAMS:
                try:
                    sh["env_params"][k] = env.get_param(k)
                except NAT.QuadSwarmError:
                    pass
        if getattr(env, "replay", None) is not None:
            sh["replay_ws"] = env._replay_ws.cpu().clone()
        return sh

    def _gather_shards(self, shard):
        """Every rank's shard on rank 0 (None elsewhere): each serialised with torch.save, the lengths all-gathered (8
        bytes per rank), the byte strings padded to the longest and gathered to rank 0 only (the other ranks hold just
        their own padded string), read back with weights_only=True."""
        if not self.distributed:
            return [shard]
        import io
        import torch.distributed as dist
        bio = io.BytesIO()
        torch.save(shard, bio)
        raw = torch.frombuffer(bytearray(bio.getvalue()), dtype=torch.uint8)
        cdev = self.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        n = torch.tensor([raw.numel()], dtype=torch.int64, device=cdev)
        ns = torch.empty(self.world_size, dtype=torch.int64, device=cdev)
        dist.all_gather_into_tensor(ns, n, group=self.group)
        ns = ns.cpu().tolist()
        pad = torch.zeros(max(ns), dtype=torch.uint8)
        pad[:raw.numel()] = raw
        pad = pad.to(cdev)
        dst = dist.get_global_rank(self.group, 0) if self.group is not None else 0
        parts = [torch.empty_like(pad) for _ in range(self.world_size)] if self.rank == 0 else None
        dist.gather(pad, gather_list=parts, dst=dst, group=self.group)
        if self.rank != 0:
            return None
        return [torch.load(io.BytesIO(parts[r][:ns[r]].cpu().numpy().tobytes()), map_location="cpu",
                           weights_only=True) for r in range(self.world_size)]

    def save(self, path, callbacks=None):
        """Everything the next iteration depends on: policy and Adam state, counters, the callbacks' state, and every
        rank's shard (_shard_state).  Collective under data parallelism: every rank calls it with the same path, rank
        0 writes ONE file holding all shards (in rank order, with the world size).  Loaded with
        torch.load(weights_only=True).  Resuming reproduces the continuation bitwise (tests/test_gpu_trainer.py,
        tests/test_trainer_distributed_cpu.py)."""
        from dataclasses import asdict
        callbacks = self.callbacks if callbacks is None else callbacks
        shards = self._gather_shards(self._shard_state())
        cbs = [cb.state_dict() for cb in callbacks]
        if self.rank == 0:
            ck = {"format": self.CKPT_FORMAT, "world_size": self.world_size,
                  "policy": self.policy.state_dict(), "optimizer": self.optimizer.state_dict(),
                  "policy_cfg": asdict(self.policy.cfg), "ppo_cfg": asdict(self.cfg),
                  "num_timesteps": self.num_timesteps, "env_steps": self.env_steps, "iterations": self.iterations,
                  "callbacks": cbs, "shards": shards}
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            tmp = path + ".tmp"
            torch.save(ck, tmp)
            os.replace(tmp, path)
        if self.distributed:   # the file exists for every rank when save() returns
            import torch.distributed as dist
            dist.barrier(group=self.group)
        return path

    def load(self, path, callbacks=()):
        """Restore a save() checkpoint into this trainer (same policy / env configuration and the same world size;
        each rank takes its own shard); `callbacks` (the same kinds, in the order they were saved) get their state
        back for the next learn()."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        if ck.get("format") != self.CKPT_FORMAT:
            raise ValueError(f"{path}: not a {self.CKPT_FORMAT} checkpoint")
        if int(ck["world_size"]) != self.world_size:
            raise ValueError(f"{path}: written by {ck['world_size']} ranks, this run has {self.world_size} "
                             "(the env shards are per rank)")
        sh = ck["shards"][self.rank]
        self.policy.load_state_dict(ck["policy"])
        self.optimizer.load_state_dict(ck["optimizer"])
        self.num_timesteps, self.env_steps, self.iterations = (int(ck["num_timesteps"]), int(ck["env_steps"]),
                                                                int(ck["iterations"]))
        self.gen.set_state(sh["gen"])
        if self.device.type == "cuda":
            torch.cuda.set_rng_state(sh["device_rng"], self.device)
        else:
            torch.set_rng_state(sh["device_rng"])
        env = self.env
        if "env_state" in sh:
            for k, v in sh.get("env_params", {}).items():
                env.set_param(k, v)
            env.set_state(bytes(sh["env_state"].numpy().tobytes()))
        if "replay_ws" in sh:
            env._replay_ws.copy_(sh["replay_ws"].to(env._replay_ws.device))
        if sh["last_obs"] is not None:
            obs = getattr(env, "obs", None)
            if obs is None:
                obs = torch.empty_like(sh["last_obs"], device=self.device)
            obs.copy_(sh["last_obs"].to(self.device))
            self.last_obs = obs
        self.last_done.copy_(sh["last_done"].to(self.device))
        self.last_values.copy_(sh["last_values"].to(self.device))
        for cb, sd in zip(callbacks, ck["callbacks"]):
            cb.load_state_dict(sd)
        if self.fused is not None:
            self.fused.refresh()
        return ck
