"""Phase timeline of the fused DAMA head kernels (csrc/head.hip built with -DEWVIT_HEAD_TRACE):
workgroup 0's wall-clock stamps (100 MHz) at every phase boundary, forward + backward at 64
frames, training mode.  Usage: python tools/head_trace.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def main():
    import ewvit
    from network.dama import DAMA
    dev = 'cuda'
    torch.manual_seed(0)
    m = DAMA(3, 128, 4, 3, 8).to(dev).train()
    s0 = torch.randn(64, 128, device=dev, requires_grad=True)
    f0 = torch.randn(64, 128, device=dev, requires_grad=True)
    for it in range(4):
        ewvit._lib.rng_advance(s0.device)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            fused, s, f = ewvit.head.dama_head(m, s0, f0, 1234)
        ws = fused.grad_fn.saved_tensors[0]
        torch.autograd.backward([fused, s, f], [torch.ones_like(fused)] * 3)
        torch.cuda.synchronize()
    st = ws[-256:].view(torch.int64).cpu().tolist()
    for name, lo, hi in (('fwd rows', 0, 32), ('fwd tail', 32, 48), ('bwd tail', 48, 64), ('bwd rows', 64, 128)):
        v = [x for x in st[lo:hi] if x > 0]
        if not v:
            continue
        d = [round((b - a) * 0.01, 2) for a, b in zip(v, v[1:])]
        print(f'{name}: total {(v[-1] - v[0]) * 0.01:.1f} us, phases (us): {d}', flush=True)


if __name__ == '__main__':
    main()
