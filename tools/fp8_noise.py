"""Spread of the fp8 DAMA forward's error against the fp32 oracle over input seeds (the
quantity tests/test_gpu_fp8.py::test_dama_train_step_fp8_vs_oracle bounds): per seed, max |err|
/ scale and cosine of the fused / space / freq outputs, train mode, same recipe weights.
Run under two builds (EWVIT_LIB) to see whether a bit-level change moves the distribution or
only the draw.  usage: python tools/fp8_noise.py [seeds...]"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'efficient-wavelet-vit_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)


def main(seeds):
    from network import dama, set_gemm_precision
    from oracle import model as om
    from oracle.weights import recipe_input
    from test_gpu_modules import pair, cos
    torch.manual_seed(0)
    p, o = pair(dama.DAMA, om.DAMA, (3, 128, 4, 3, 8), 14)
    set_gemm_precision(p, 'fp8')
    p.train(); o.train()
    for s in seeds:
        x = recipe_input((2, 8, 3, 224, 224), seed=s)
        with torch.no_grad():
            ro = o(x, batch_size=4)
            with torch.autocast('cuda', dtype=torch.bfloat16):
                rp = p(x.to('cuda'), batch_size=4)
        row = {'seed': s}
        for k in sorted(ro):
            a, b = rp[k].detach().float().cpu(), ro[k].detach().float()
            row[k] = (round(float((a - b).abs().max()) / max(float(b.abs().max()), 1e-6), 4), round(cos(a, b), 5))
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main([int(a) for a in sys.argv[1:]] or [4242, 1, 2, 3, 4, 5, 6, 7])
