#!/usr/bin/env python
"""Policy fixtures from the reference's own model code (TEST INFRASTRUCTURE, dev container only).

    python tools/gen_golden_policy.py       # writes tests/golden/policy_<case>.npz + policy_<case>.json

Builds the reference's `ActorCriticPolicyCustomSeparateWeights` (swarm_rl/models/ActorCriticPolicyCustom.py:284-554)
with its `QuadMultiEncoder` / `QuadNeighborhoodEncoder{Attention,Deepsets,Mlp}` (swarm_rl/models/
quad_multi_model.py:24-122, 250-353) and `ModelCoreMLP` (ActorCriticPolicyCustom.py:260-281), imported from
/root/reference through tools/refshim.py.  Their third-party bases are not installed, so this script adds
stand-ins restating the published behaviour the reference calls (parity unpinned for these pieces):
  sample_factory 2.x   fc_layer = nn.Linear, nonlinearity(cfg) = Tanh/ReLU/ELU, Encoder/ModelCore = nn.Module
                       holding cfg, calc_num_elements = numel of the module's output on a (1, *shape) torch.rand
                       input, ModelCoreIdentity (passes features through), MlpDecoder (create_mlp; nn.Identity for
                       decoder_mlp_layers = [])
  stable_baselines3    ActorCriticPolicy (nn.Module base; `device` = the parameters' device), and
                       SquashedDiagGaussianDistribution: proba_distribution_net = (Linear(latent, A), log_std
                       Parameter), log_prob(a) = Normal(mean, exp(log_std)).log_prob(atanh(clamp(a, +-(1-eps))))
                       summed - sum log(1 - a^2 + 1e-6), mode = tanh(mean), entropy = None
Every parameter is then set from tests/policy_fixture.param_value(reference name, shape), so the fixture holds
the reference's parameter names and shapes, the inputs and the outputs -- no weight arrays, no reference source.

Recorded per case:
  fp64  each tower's neighbour encoder output (quad_multi_model.py:73-101 incl. the Tensor.repeat row pairing)
        and QuadMultiEncoder output, called on {'obs': obs64} directly
  fp32  the policy's forward(obs, deterministic=True) -> actions, values, log_prob and
        evaluate_actions(obs, actions) -> values, log_prob (prepare_obs casts to float32, :462-470)
"""
import json
import os
import sys
import textwrap
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import refshim  # noqa: E402

import torch  # noqa: E402
from policy_fixture import param_value  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

_EXTRA = {
    "sample_factory/algo/__init__.py": "",
    "sample_factory/algo/utils/__init__.py": "",
    "sample_factory/algo/utils/context.py": """
        class _Factory:
            def register_encoder_factory(self, f): self.encoder_factory = f
        _F = _Factory()
        def global_model_factory(): return _F
    """,
    "sample_factory/algo/utils/torch_utils.py": """
        import torch
        def calc_num_elements(module, module_input_shape):
            return module(torch.rand((1,) + tuple(module_input_shape))).numel()
    """,
    "sample_factory/algo/utils/action_distributions.py": """
        def is_continuous_action_space(space): return True
        def sample_actions_log_probs(distribution): raise NotImplementedError
    """,
    "sample_factory/model/__init__.py": "",
    "sample_factory/model/model_utils.py": """
        from torch import nn
        def fc_layer(in_features, out_features, bias=True, spec_norm=False):
            return nn.Linear(in_features, out_features, bias)
        def nonlinearity(cfg, inplace=False):
            if cfg.nonlinearity == "elu": return nn.ELU(inplace=inplace)
            if cfg.nonlinearity == "relu": return nn.ReLU(inplace=inplace)
            if cfg.nonlinearity == "tanh": return nn.Tanh()
            raise Exception("Unknown nonlinearity")
    """,
    "sample_factory/model/encoder.py": """
        from torch import nn
        class Encoder(nn.Module):
            def __init__(self, cfg):
                super().__init__()
                self.cfg = cfg
    """,
    "sample_factory/model/core.py": """
        from torch import nn
        class ModelCore(nn.Module):
            def __init__(self, cfg):
                super().__init__()
                self.cfg = cfg
                self.core_output_size = -1
            def get_out_size(self): return self.core_output_size
        class ModelCoreIdentity(ModelCore):
            def __init__(self, cfg, input_size):
                super().__init__(cfg)
                self.core_output_size = input_size
            def forward(self, head_output, fake_rnn_states): return head_output, fake_rnn_states
        def default_make_core_func(cfg, core_input_size): return ModelCoreIdentity(cfg, core_input_size)
    """,
    "sample_factory/model/decoder.py": """
        from torch import nn
        from sample_factory.model.model_utils import nonlinearity
        from sample_factory.algo.utils.torch_utils import calc_num_elements
        def create_mlp(layer_sizes, input_size, activation):
            layers = []
            for size in layer_sizes:
                layers.extend([nn.Linear(input_size, size), activation])
                input_size = size
            return nn.Sequential(*layers) if layers else nn.Identity()
        class MlpDecoder(nn.Module):
            def __init__(self, cfg, decoder_input_size):
                super().__init__()
                self.cfg = cfg
                self.mlp = create_mlp(cfg.decoder_mlp_layers, decoder_input_size, nonlinearity(cfg))
                self.decoder_out_size = calc_num_elements(self.mlp, (decoder_input_size,))
            def forward(self, core_output): return self.mlp(core_output)
            def get_out_size(self): return self.decoder_out_size
    """,
    "sample_factory/model/action_parameterization.py": """
        class ActionParameterizationContinuousNonAdaptiveStddev: pass
        class ActionParameterizationDefault: pass
    """,
    "sample_factory/utils/typing.py": "from typing import Any\nConfig = Any\n",
    "sample_factory/utils/normalize.py": "class ObservationNormalizer: pass\n",
    "stable_baselines3/__init__.py": "",
    "stable_baselines3/common/__init__.py": "",
    "stable_baselines3/common/torch_layers.py": "from torch import nn\nclass BaseFeaturesExtractor(nn.Module): pass\n",
    "stable_baselines3/common/policies.py": """
        import torch
        from torch import nn
        class ActorCriticPolicy(nn.Module):
            def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, **kwargs):
                super().__init__()
                self.observation_space, self.action_space = observation_space, action_space
            @property
            def device(self):
                for p in self.parameters():
                    return p.device
                return torch.device("cpu")
    """,
    "stable_baselines3/common/distributions.py": """
        import torch as th
        from torch import nn
        from torch.distributions import Normal
        class Distribution: pass
        class BernoulliDistribution(Distribution): pass
        class CategoricalDistribution(Distribution): pass
        class MultiCategoricalDistribution(Distribution): pass
        class StateDependentNoiseDistribution(Distribution): pass
        def make_proba_distribution(*a, **k): raise NotImplementedError
        def sum_independent_dims(t): return t.sum(dim=1) if len(t.shape) > 1 else t.sum()
        class DiagGaussianDistribution(Distribution):
            def __init__(self, action_dim):
                self.action_dim = action_dim
            def proba_distribution_net(self, latent_dim, log_std_init=0.0):
                return nn.Linear(latent_dim, self.action_dim), nn.Parameter(th.ones(self.action_dim) * log_std_init)
            def proba_distribution(self, mean_actions, log_std):
                self.distribution = Normal(mean_actions, th.ones_like(mean_actions) * log_std.exp())
                return self
            def log_prob(self, actions): return sum_independent_dims(self.distribution.log_prob(actions))
            def entropy(self): return sum_independent_dims(self.distribution.entropy())
            def mode(self): return self.distribution.mean
            def sample(self): return self.distribution.rsample()
            def get_actions(self, deterministic=False): return self.mode() if deterministic else self.sample()
        def _atanh(x): return 0.5 * (x.log1p() - (-x).log1p())
        class SquashedDiagGaussianDistribution(DiagGaussianDistribution):
            def __init__(self, action_dim, epsilon=1e-6):
                super().__init__(action_dim)
                self.epsilon = epsilon
            def log_prob(self, actions, gaussian_actions=None):
                if gaussian_actions is None:
                    eps = th.finfo(actions.dtype).eps
                    gaussian_actions = _atanh(actions.clamp(min=-1.0 + eps, max=1.0 - eps))
                lp = super().log_prob(gaussian_actions)
                return lp - th.sum(th.log(1 - actions ** 2 + self.epsilon), dim=1)
            def entropy(self): return None
            def mode(self): return th.tanh(super().mode())
            def sample(self): return th.tanh(super().sample())
    """,
}


def install():
    d = refshim.install()
    for rel, src in _EXTRA.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(src))
    for m in [m for m in sys.modules if m.startswith("sample_factory")]:
        del sys.modules[m]


# (reference cfg fields, act_dim, batch): the configs this repository runs the policy at
CASES = {
    # C3 (bench e2e, flavor B): xyz_vxyz_R_omega 18 + pos_vel 6 x 6, attention 256, identity core
    "c3": (dict(obs_repr="xyz_vxyz_R_omega", neighbor_obs_type="pos_vel", neighbor_visible_num=6, num_agents=8,
                neighbor_encoder_type="attention", neighbor_hidden_size=256, rnn_size=256, rnn_type="none",
                rnn_num_layers=0), 4, 67),
    # sb_train (flavor A, sb_train.py:111-137 / global_cfg.py): 7 + ndist_nsangle 3 x 7, attention 128, 6 x 128 core
    "a8": (dict(obs_repr="cdist_cdistdot_ndist_distdot_nsangle_angledot", neighbor_obs_type="ndist_nsangle",
                neighbor_visible_num=-1, num_agents=8, neighbor_encoder_type="attention", neighbor_hidden_size=128,
                rnn_size=128, rnn_type="full", rnn_num_layers=6), 2, 45),
    # C4: floor repr 19 + pos_vel 6 x 2 + octomap SDF 9, obstacle encoder
    "c4": (dict(obs_repr="xyz_vxyz_R_omega_floor", neighbor_obs_type="pos_vel", neighbor_visible_num=2, num_agents=8,
                neighbor_encoder_type="attention", neighbor_hidden_size=256, rnn_size=256, rnn_type="none",
                rnn_num_layers=0, use_obstacles=True, obstacle_obs_type="octomap", obst_hidden_size=256), 4, 33),
    "mean_embed": (dict(obs_repr="xyz_vxyz_R_omega", neighbor_obs_type="pos_vel", neighbor_visible_num=-1,
                        num_agents=4, neighbor_encoder_type="mean_embed", neighbor_hidden_size=64, rnn_size=64,
                        rnn_type="full", rnn_num_layers=2), 4, 21),
    "mlp": (dict(obs_repr="cdist_cdistdot_dist_distdot_sangle_angledot", neighbor_obs_type="dist_sangle",
                 neighbor_visible_num=3, num_agents=8, neighbor_encoder_type="mlp", neighbor_hidden_size=64,
                 rnn_size=64, rnn_type="none", rnn_num_layers=0), 2, 19),
}


def ref_cfg(fields):
    c = dict(use_obstacles=False, obstacle_obs_type="none", obst_hidden_size=256, nonlinearity="tanh",
             policy_init_gain=1.0, decoder_mlp_layers=[])
    c.update(fields)
    return types.SimpleNamespace(**c)


def main():
    install()
    from gymnasium import spaces
    from gym_art.quadrotor_multi.quad_utils import QUADS_NEIGHBOR_OBS_TYPE, QUADS_OBS_REPR, QUADS_OBSTACLE_OBS_TYPE
    from swarm_rl.models.ActorCriticPolicyCustom import ActorCriticPolicyCustomSeparateWeights

    for case, (fields, act_dim, B) in CASES.items():
        cfg = ref_cfg(fields)
        k = cfg.num_agents - 1 if cfg.neighbor_visible_num == -1 else cfg.neighbor_visible_num
        so = QUADS_OBS_REPR[cfg.obs_repr]
        nd = QUADS_NEIGHBOR_OBS_TYPE[cfg.neighbor_obs_type]
        od = so + nd * k + (QUADS_OBSTACLE_OBS_TYPE[cfg.obstacle_obs_type] if cfg.use_obstacles else 0)
        torch.manual_seed(0)
        obs_space = spaces.Box(-np.ones(od), np.ones(od))
        act_space = spaces.Box(-np.ones(act_dim), np.ones(act_dim))
        pol = ActorCriticPolicyCustomSeparateWeights(obs_space, act_space, lambda _: 1e-4, cfg)
        names, shapes = [], []
        with torch.no_grad():
            for n, p in pol.named_parameters():
                p.copy_(param_value(n, p.shape, p.dtype))
                names.append(n)
                shapes.append(list(p.shape))
        rng = np.random.default_rng(sum(map(ord, case)))
        obs = rng.normal(0.0, 1.5, (B, od))
        act = rng.uniform(-0.95, 0.95, (B, act_dim))
        out = {"obs": obs, "act": act}
        pol64 = pol.double()
        with torch.no_grad():
            o64 = torch.from_numpy(obs)
            for tw in ("actor", "critic"):
                enc = getattr(pol64, f"{tw}_encoder")
                out[f"{tw}_features64"] = enc({"obs": o64}).numpy()
                if enc.neighbor_encoder is not None:
                    out[f"{tw}_nbr64"] = enc.neighbor_encoder(o64[:, :so], o64, enc.all_neighbor_obs_size, B).numpy()
        pol32 = pol.float()
        with torch.no_grad():
            o32 = torch.from_numpy(obs.astype(np.float32))
            a, v, lp = pol32.forward(o32, deterministic=True)
            out.update(det_actions32=a.numpy(), det_values32=v.numpy(), det_log_prob32=lp.numpy())
            v2, lp2, ent = pol32.evaluate_actions(o32, torch.from_numpy(act.astype(np.float32)))
            assert ent is None
            out.update(eval_values32=v2.numpy(), eval_log_prob32=lp2.numpy())
            out["pv_values32"] = pol32.predict_values(o32).numpy()
        np.savez_compressed(os.path.join(OUT, f"policy_{case}.npz"), **out)
        meta = {"case": case, "ref_cfg": vars(cfg), "act_dim": act_dim, "batch": B, "obs_dim": od,
                "self_obs_dim": so, "neighbor_obs_dim": nd, "num_use_neighbor_obs": k,
                "param_names": names, "param_shapes": shapes,
                "param_count": int(sum(int(np.prod(s)) for s in shapes))}
        with open(os.path.join(OUT, f"policy_{case}.json"), "w") as f:
            json.dump(meta, f, indent=1)
        print(case, od, meta["param_count"], len(names))


if __name__ == "__main__":
    main()
