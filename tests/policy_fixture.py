"""Deterministic policy weights for the reference-generated policy fixtures (TEST INFRASTRUCTURE).

tools/gen_golden_policy.py builds the reference's own ActorCriticPolicyCustomSeparateWeights
(swarm_rl/models/ActorCriticPolicyCustom.py:284-554) and sets every parameter from `param_value(name, shape)`,
keyed by the reference's parameter name; the tests rebuild the same tensors from the names recorded in the
fixture, so the fixture holds names, inputs and outputs only (no weight arrays).  The scale is widened beyond
PyTorch's default Linear init (2 / sqrt(fan_in), biases +-0.3) so every tanh runs in its nonlinear range and
the attention softmax is far from uniform."""
import zlib

import torch


def param_value(name, shape, dtype=torch.float64):
    g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
    u = torch.rand(tuple(shape), generator=g, dtype=torch.float64) * 2.0 - 1.0
    if name.endswith("log_std"):
        return torch.full(tuple(shape), -0.7, dtype=dtype)
    if len(shape) == 2:
        return (u * (2.0 / shape[1] ** 0.5)).to(dtype)
    return (u * 0.3).to(dtype)


def state_dict_from_names(names, shapes, dtype=torch.float64):
    return {n: param_value(n, s, dtype) for n, s in zip(names, shapes)}
