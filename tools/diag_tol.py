"""Diagnostic (GPU): where the DAMA train-step error against the fp32 oracle comes from,
to set fixed parity bounds.  For chunk sizes of 8 and 16 frames it prints, per output and
per parameter gradient, the product's error / cosine, torch bf16 autocast's (the oracle
moved to the GPU), and torch fp32 on the GPU (the oracle itself on the GPU: CPU/GPU fp32
agreement).  Output: gpurun_out/diag_tol.json (+ stdout)."""
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
    from network import dama
    from oracle import model as om
    from oracle.weights import recipe_input
    torch.manual_seed(0)
    p0, o0 = T.pair(dama.DAMA, om.DAMA, (3, 128, 4, 3, 8), 14)
    res = {}
    for per_video in (4, 8):
        x = recipe_input((2, 8, 3, 224, 224) if per_video == 4 else (2, 16, 3, 224, 224), seed=4242)
        o = copy.deepcopy(o0).train()
        ro = o(x, batch_size=per_video)
        w = {k: torch.randn(v.shape, generator=torch.Generator().manual_seed(i))
             for i, (k, v) in enumerate(sorted(ro.items()))}
        sum((ro[k] * w[k]).sum() for k in ro).backward()
        oo = dict(o.named_parameters())
        names = [n for n, q in oo.items() if q.grad is not None]

        def variant(model, autocast):
            model.train()
            with torch.autocast('cuda', dtype=torch.bfloat16, enabled=autocast):
                r = model(x.cuda(), batch_size=per_video)
            sum((r[k].float() * w[k].cuda()).sum() for k in r).backward()
            pp = dict(model.named_parameters())
            out = {'fwd_err_of_scale': {k: float((r[k].float().cpu() - ro[k]).abs().max() / ro[k].abs().max())
                                        for k in r},
                   'fwd_cos': {k: T.cos(r[k], ro[k]) for k in r},
                   'grad_cos': {n: T.cos(pp[n].grad, oo[n].grad) for n in names if pp[n].grad is not None}}
            gc = sorted(out['grad_cos'].items(), key=lambda kv: kv[1])
            out['grad_cos_worst'] = gc[:12]
            return out
        v = {'product': variant(copy.deepcopy(p0), True),
             'torch_autocast_bf16': variant(copy.deepcopy(o0).cuda(), True),
             'torch_fp32_gpu': variant(copy.deepcopy(o0).cuda(), False)}
        res[f'chunk{2 * per_video}'] = v
        for name, d in v.items():
            print(f'== chunk {2 * per_video} {name}: fwd err ' +
                  ', '.join(f'{k} {e:.4f}/cos {d["fwd_cos"][k]:.6f}' for k, e in d['fwd_err_of_scale'].items()))
            for n, c in d['grad_cos_worst']:
                print(f'   {n:60s} {c:.5f}')
            fg = d['grad_cos'].get('fusion_gate.0.weight')
            print(f'   fusion_gate.0.weight {fg}')
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    json.dump(res, open(os.path.join(REPO, 'gpurun_out', 'diag_tol.json'), 'w'), indent=1)


if __name__ == '__main__':
    main()
