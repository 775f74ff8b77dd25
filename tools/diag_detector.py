"""Diagnostic (GPU): the DeepfakeDetector train-step outputs (one 8-frame chunk, train-mode
BatchNorm) against the fp32 oracle over several input seeds — the product (ewvit stem on
and off) and torch's own bf16 autocast of the oracle — to set the detector test's fixed
output bound from a distribution.  Output: gpurun_out/diag_detector.json (+ stdout)."""
import copy
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'efficient-wavelet-vit_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)

import test_gpu_modules as T  # noqa: E402


def main():
    import network.efficientnet as en
    from network.model import DeepfakeDetector
    from oracle import model as om
    from oracle.weights import recipe_input, recipe_state_dict
    p0 = DeepfakeDetector(3, 128, batch_size=4)
    sd = recipe_state_dict(p0.state_dict(), 15)
    p0.load_state_dict(sd)
    p0 = T.no_stochastic(p0)
    o0 = T.no_stochastic(om.DeepfakeDetector(3, 128, batch_size=4))
    o0.load_state_dict(recipe_state_dict(o0.state_dict(), 15))   # the recipe is keyed by name
    res = {}
    for seed in [int(s) for s in os.environ.get('SEEDS', '1008 1 2 3').split()]:
        x = recipe_input((2, 4, 3, 224, 224), seed=seed)
        ro = copy.deepcopy(o0).train()(x, 4, 'dynamic')

        def variant(model):
            model.train()
            with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):
                r = model(x.cuda(), 4, 'dynamic')
            return {k: float((r[k].float().cpu() - ro[k].detach()).abs().max() / ro[k].detach().abs().max())
                    for k in ('fused', 'space', 'freq', 'logits')}
        en._STEM = True
        v = {'product_stem': variant(copy.deepcopy(p0).cuda().to(memory_format=torch.channels_last))}
        en._STEM = False
        v['product_libstem'] = variant(copy.deepcopy(p0).cuda().to(memory_format=torch.channels_last))
        en._STEM = True
        v['torch_autocast_bf16'] = variant(copy.deepcopy(o0).cuda())
        res[seed] = v
        print(f'== seed {seed}', flush=True)
        for n, d in v.items():
            print(f'   {n:22s} ' + '  '.join(f'{k} {e:.4f}' for k, e in d.items()), flush=True)
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(REPO, 'gpurun_out', 'diag_detector.json'), 'w') as f:
        json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
