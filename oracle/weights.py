"""ORACLE (test infrastructure only) — a portable, deterministic weight recipe.

The reference initialises from torch's global RNG in module-construction order,
which no independent implementation can reproduce.  Parity fixtures therefore
overwrite every parameter/buffer from this recipe, which depends only on the
state-dict key, its shape and a seed:

    rng   = numpy.random.default_rng([seed, crc32(key)])
    value = standard_normal(shape) * scale(key, shape)   (float32)

* weights: scale = 1/sqrt(fan_in) (fan_in = prod(shape[1:]), or 1)
* biases / LayerNorm & BatchNorm bias / running_mean: scale 0.05
* LayerNorm/BatchNorm weight: 1 + 0.1*N(0,1)
* BatchNorm running_var: 1 + 0.2*|N(0,1)|
* pos_embedding / cls_token: N(0,1) (their reference init is torch.randn)
* num_batches_tracked: 0
"""
import zlib

import numpy as np
import torch


def recipe_tensor(key, shape, seed=0):
    rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
    n = rng.standard_normal(size=tuple(shape)).astype(np.float32)
    leaf = key.rsplit('.', 1)[-1]
    if leaf == 'num_batches_tracked':
        return np.zeros(shape, dtype=np.int64)
    if leaf == 'running_var':
        return (1.0 + 0.2 * np.abs(n)).astype(np.float32)
    if leaf == 'running_mean':
        return (0.05 * n).astype(np.float32)
    if key.endswith('pos_embedding') or key.endswith('cls_token'):
        return n
    if leaf.startswith('h0_') or leaf.startswith('h1_'):
        return None  # fixed DWT filter buffers: keep
    if leaf == 'bias':
        return (0.05 * n).astype(np.float32)
    if leaf == 'weight' and len(shape) == 1:          # LayerNorm / BatchNorm affine
        return (1.0 + 0.1 * n).astype(np.float32)
    fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    return (n / np.sqrt(max(fan_in, 1))).astype(np.float32)


def recipe_state_dict(state_dict, seed=0):
    out = {}
    for k, v in state_dict.items():
        t = recipe_tensor(k, tuple(v.shape), seed)
        out[k] = v.clone() if t is None else torch.from_numpy(t).to(v.dtype)
    return out


def apply_recipe(module, seed=0):
    module.load_state_dict(recipe_state_dict(module.state_dict(), seed))
    return module


def recipe_input(shape, seed=1000):
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(size=shape).astype(np.float32))
