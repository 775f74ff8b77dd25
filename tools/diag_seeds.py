"""Diagnostic (GPU): spread of the DAMA train-step gradient cosines against the fp32 oracle
over several input seeds — the product (stem on the ewvit direct conv, and on the library
conv) and torch's own bf16 autocast of the oracle — for the layers test_gpu_modules bounds
(GRAD_FLOOR) plus the mean / min over all non-bias weights.  Sets the fixed floors from a
distribution rather than one draw.  Output: gpurun_out/diag_seeds.json (+ stdout)."""
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
    from network import dama
    from oracle import model as om
    from oracle.weights import recipe_input
    torch.manual_seed(0)
    p0, o0 = T.pair(dama.DAMA, om.DAMA, (3, 128, 4, 3, 8), 14)
    seeds = [int(s) for s in os.environ.get('SEEDS', '4242 1 2 3').split()]
    res = {}
    for seed in seeds:
        x = recipe_input((2, 8, 3, 224, 224), seed=seed)
        o = copy.deepcopy(o0).train()
        ro = o(x, batch_size=4)
        w = {k: torch.randn(v.shape, generator=torch.Generator().manual_seed(i))
             for i, (k, v) in enumerate(sorted(ro.items()))}
        sum((ro[k] * w[k]).sum() for k in ro).backward()
        oo = dict(o.named_parameters())
        names = [n for n, q in oo.items() if q.grad is not None and not n.endswith('.bias')]

        def variant(model):
            model.train()
            with torch.autocast('cuda', dtype=torch.bfloat16):
                r = model(x.cuda(), batch_size=4)
            sum((r[k].float() * w[k].cuda()).sum() for k in r).backward()
            pp = dict(model.named_parameters())
            gc = {n: T.cos(pp[n].grad, oo[n].grad) for n in names if pp[n].grad is not None}
            out = {k: gc[k] for k in T.GRAD_FLOOR}
            out['_mean'] = sum(gc.values()) / len(gc)
            worst = min(gc.items(), key=lambda kv: kv[1])
            out['_min'] = worst[1]
            out['_min_name'] = worst[0]
            out['_fwd_err'] = {k: float((r[k].float().cpu() - ro[k]).abs().max() / ro[k].abs().max()) for k in r}
            return out
        en._STEM = True
        v = {'product_stem': variant(copy.deepcopy(p0))}
        en._STEM = False
        v['product_libstem'] = variant(copy.deepcopy(p0))
        en._STEM = True
        v['torch_autocast_bf16'] = variant(copy.deepcopy(o0).cuda())
        res[seed] = v
        print(f'== seed {seed}', flush=True)
        for k in list(T.GRAD_FLOOR) + ['_mean', '_min']:
            print(f'   {k:55s} ' + '  '.join(f'{n} {d[k]:.4f}' for n, d in v.items()), flush=True)
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(REPO, 'gpurun_out', 'diag_seeds.json'), 'w') as f:
        json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
