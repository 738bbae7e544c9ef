"""Range guards of the split-f16 (x3) rollout encoders: weights beyond f16's range at the
packing scale are refused by the packer, FusedRolloutPolicy packs fp32 instead (and back to x3 once the weights are
in range), and observations beyond the layer-0 scale's range make check_inputs() raise.  Host-side packing only
(no kernel launch)."""
import warnings

import pytest
import torch

from quadswarm_amd.policy_fused import F16_MAX, X3_SIN, X3_SW, FusedRolloutPolicy, pack_mfma_weight_x3
from quadswarm_amd.ppo import SwarmActorCritic
from test_ppo_cpu import sb_cfg


def test_pack_x3_refuses_out_of_range_weights():
    w = torch.randn(32, 32) * 0.1
    pack_mfma_weight_x3(w)
    w[3, 7] = F16_MAX / X3_SW * 1.001
    with pytest.raises(ValueError, match="split-f16 range"):
        pack_mfma_weight_x3(w)
    w[3, 7] = float("nan")
    with pytest.raises(ValueError):
        pack_mfma_weight_x3(w)


def test_fused_policy_falls_back_to_fp32_packing_and_back():
    torch.manual_seed(0)
    pol = SwarmActorCritic(sb_cfg()[1])
    f = FusedRolloutPolicy(pol, precision="x3")
    f.refresh()
    assert f.packed_precision == "x3"
    ne = pol.actor_encoder.neighbor_encoder
    with torch.no_grad():
        old = ne.attention_mlp[2].weight[0, 0].item()
        ne.attention_mlp[2].weight[0, 0] = 300.0
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        f.refresh()
    assert f.packed_precision == "fp32" and any("f16 range" in str(r.message) for r in rec)
    assert f.packed[0]["w_a2p"].dtype == torch.float32
    with torch.no_grad():
        ne.attention_mlp[2].weight[0, 0] = old
    f.refresh()
    assert f.packed_precision == "x3" and f.packed[0]["w_a2p"].dtype == torch.int16


def test_check_inputs_raises_on_out_of_range_observations():
    pol = SwarmActorCritic(sb_cfg()[1])
    f = FusedRolloutPolicy(pol, precision="x3")
    f.check_inputs()                                    # nothing recorded
    f._obs_absmax = torch.tensor(F16_MAX / X3_SIN * 0.99)
    f.check_inputs()
    f._obs_absmax = torch.tensor(float("nan"))          # non-finite obs: the env's guard reports those
    f.check_inputs()
    f._obs_absmax = torch.tensor(F16_MAX / X3_SIN)
    with pytest.raises(ValueError, match="rollout_precision='fp32'"):
        f.check_inputs()
    assert f._obs_absmax is None                        # reset after every check


def test_fused_update_observation_range_guard():
    """the fused x3 update checks the rollout's observations once per update (PPOTrainer.train) and
    runs that update's encoders on the torch path when one is beyond layer 0's split-f16 range."""
    from quadswarm_amd.encoder_train import FusedAttentionTrain
    pol = SwarmActorCritic(sb_cfg()[1])
    f = FusedAttentionTrain(pol)
    obs = torch.randn(64, 28)
    assert f.obs_in_range(obs)
    obs[5, 3] = -F16_MAX / X3_SIN
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        assert not f.obs_in_range(obs)
    assert any("torch fp32" in str(r.message) for r in rec)
    obs[5, 3] = float("nan")                           # non-finite: the env's guard reports those
    assert f.obs_in_range(obs)
