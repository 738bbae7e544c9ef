"""The policy mirror (quadswarm_amd.ppo.SwarmActorCritic) against the reference's own policy module.

tests/golden/policy_<case>.{npz,json} come from tools/gen_golden_policy.py, which builds the reference's
ActorCriticPolicyCustomSeparateWeights (swarm_rl/models/ActorCriticPolicyCustom.py:284-554) with its
QuadMultiEncoder / neighbour encoders (swarm_rl/models/quad_multi_model.py:24-122, 250-353) and ModelCoreMLP
(:260-281), sets every parameter from tests/policy_fixture.param_value(name, shape), and records the outputs.
Here the same weights, keyed by the reference's names, are loaded into SwarmActorCritic through
load_reference_state_dict (the checkpoint-interchange path) and the outputs compared:
  fp64  neighbour encoder and QuadMultiEncoder outputs of both towers within 1e-12 (the split evaluation of the
        concatenating layers, ppo.NeighborAttention.split, differs from the reference's torch.cat GEMM only in
        summation order);
  fp32  forward(deterministic) actions / values / log-probs and evaluate_actions within fp32 summation order.
The sample_factory layers (fc_layer, nonlinearity, MlpDecoder) and SB3's SquashedDiagGaussianDistribution the
reference calls are not installed here; the generator restates their published behaviour, so those pieces stay
parity-unpinned (the module composition, row pairing, concatenation orders and parameter names are pinned)."""
import json
import os

import numpy as np
import pytest
import torch

from policy_fixture import state_dict_from_names
from quadswarm_amd.ppo import PolicyConfig, SwarmActorCritic

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["c3", "a8", "c4", "mean_embed", "mlp"]


def load_case(case):
    with open(os.path.join(GOLDEN, f"policy_{case}.json")) as f:
        meta = json.load(f)
    data = dict(np.load(os.path.join(GOLDEN, f"policy_{case}.npz"), allow_pickle=False))
    rc = meta["ref_cfg"]
    pc = PolicyConfig(self_obs_dim=meta["self_obs_dim"], neighbor_obs_dim=meta["neighbor_obs_dim"],
                      num_use_neighbor_obs=meta["num_use_neighbor_obs"],
                      obstacle_obs_dim=meta["obs_dim"] - meta["self_obs_dim"]
                      - meta["neighbor_obs_dim"] * meta["num_use_neighbor_obs"],
                      rnn_size=rc["rnn_size"], rnn_type=rc["rnn_type"], rnn_num_layers=rc["rnn_num_layers"],
                      neighbor_hidden_size=rc["neighbor_hidden_size"],
                      neighbor_encoder_type=rc["neighbor_encoder_type"], obst_hidden_size=rc["obst_hidden_size"],
                      nonlinearity=rc["nonlinearity"], decoder_mlp_layers=rc["decoder_mlp_layers"],
                      act_dim=meta["act_dim"])
    return meta, data, pc


def reference_weights(meta, dtype):
    """the fixture's weights: fp32 values (the reference module is built in fp32, then .double()-ed for fp64)"""
    sd = state_dict_from_names(meta["param_names"], meta["param_shapes"], torch.float32)
    return {k: v.to(dtype) for k, v in sd.items()}


@pytest.mark.parametrize("case", CASES)
def test_parameter_names_and_shapes_match_reference(case):
    meta, _, pc = load_case(case)
    pol = SwarmActorCritic(pc)
    ours = {SwarmActorCritic.reference_key(k): list(v.shape) for k, v in pol.named_parameters()}
    want = dict(zip(meta["param_names"], meta["param_shapes"]))
    assert ours == want
    assert sum(p.numel() for p in pol.parameters()) == meta["param_count"]
    # the exported names round-trip
    assert set(pol.reference_state_dict()) == set(want)


@pytest.mark.parametrize("case", CASES)
def test_encoders_match_reference_fp64(case):
    meta, data, pc = load_case(case)
    pol = SwarmActorCritic(pc).double()
    pol.load_reference_state_dict(reference_weights(meta, torch.float64))
    obs = torch.from_numpy(data["obs"])
    so, K = pc.self_obs_dim, pc.num_use_neighbor_obs
    with torch.no_grad():
        for tw in ("actor", "critic"):
            enc = getattr(pol, f"{tw}_encoder")
            if f"{tw}_nbr64" in data:
                nbr = obs[:, so:so + K * pc.neighbor_obs_dim].reshape(obs.shape[0], K, -1)
                got = enc.neighbor_encoder(obs[:, :so], nbr).numpy()
                want = data[f"{tw}_nbr64"]
                assert np.abs(want).max() > 0.05
                np.testing.assert_allclose(got, want, rtol=0, atol=1e-12)
            np.testing.assert_allclose(enc(obs).numpy(), data[f"{tw}_features64"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("case", CASES)
def test_policy_outputs_match_reference_fp32(case):
    meta, data, pc = load_case(case)
    pol = SwarmActorCritic(pc)
    pol.load_reference_state_dict(reference_weights(meta, torch.float32))
    obs = torch.from_numpy(data["obs"].astype(np.float32))
    act = torch.from_numpy(data["act"].astype(np.float32))
    with torch.no_grad():
        a, v, lp = pol(obs, deterministic=True)
        np.testing.assert_allclose(a.numpy(), data["det_actions32"], rtol=0, atol=2e-5)
        np.testing.assert_allclose(v.numpy(), data["det_values32"], rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(lp.numpy(), data["det_log_prob32"], rtol=1e-5, atol=2e-4)
        v2, lp2, ent = pol.evaluate_actions(obs, act)
        assert ent is None
        np.testing.assert_allclose(v2.numpy(), data["eval_values32"], rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(lp2.numpy(), data["eval_log_prob32"], rtol=1e-5, atol=2e-4)
        np.testing.assert_allclose(pol.predict_values(obs).numpy(), data["pv_values32"], rtol=1e-5, atol=2e-5)


def test_row_pairing_is_batch_dependent_like_the_reference():
    """quad_multi_model.py:84-91 tiles the self obs with Tensor.repeat(K, 1) (row j -> agent j % B), so an agent's
    encoding depends on the rest of its batch: evaluating the first half of the fixture batch alone differs."""
    meta, data, pc = load_case("c3")
    pol = SwarmActorCritic(pc).double()
    pol.load_reference_state_dict(reference_weights(meta, torch.float64))
    obs = torch.from_numpy(data["obs"])
    with torch.no_grad():
        half = pol.actor_encoder(obs[:30]).numpy()
    assert np.abs(half - data["actor_features64"][:30]).max() > 1e-3
