"""Which branch bounds the config-2 step: each piece of the DAMA training step (forward +
backward, no optimizer) replayed alone from a HIP graph, timed with events over N replays.

  mwt        the MWT branch alone, on the whole chip (uncapped)
  mwt_cap    the MWT branch alone under the grid cap the step runs it with (EWVIT_MWT_GRID_CAP)
  sfe        the SFE branch (EfficientNetV2-S backbone + ViT head) alone
  full       the whole DeepfakeDetector forward + combined_loss + backward (both streams)
  step       `full` + Adam (the bench's TrainStep)
  backbone   the EfficientNetV2-S features alone
  tokens     the token path alone: sfe.head (patch_to_embedding, CLS/pos, ViT) on a fixed
             backbone map, then the step's own DAMA head (the fused cross-attention / gates
             launch when fusable), classifier and combined_loss, fwd + bwd
  probe      (--probe-us U) the step with a U-us spin kernel on the main stream right before
             the cross-attention: how much of a forward token-path microsecond the step pays

Usage: python tools/branch_time.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


class _NoOpt:
    """No update; zero_grad drops the gradients like the real optimizer (else every replay
    would add into .grad: ~480 accumulation kernels in the SFE piece)."""

    def __init__(self, params=()):
        self.params = list(params)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def step(self):
        pass


def _time(step, reps):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        step()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--tables', type=int, default=0, help='also print per-entry tables (N top launch configs)')
    ap.add_argument('--probe-us', type=float, default=0.0)
    args = ap.parse_args()
    import bench
    import ewvit
    from ewvit.graph import TrainStep
    from network.dama import _mwt_grid_cap
    dev = torch.device('cuda', 0)
    full = bench.build_step(dev, 64, 0, graph=True, config=2)
    model = full.model
    x = torch.randn(64, 3, 224, 224, device=dev)
    out = {'step_ms': _time(full, args.reps)}
    for p in model.parameters():
        p.grad = None

    def piece(fn):
        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                y = fn()
            return y.float().square().mean()
        return TrainStep(model, fl, _NoOpt(model.parameters()), graph=True)
    dama = model.dama
    out['mwt_ms'] = _time(piece(lambda: dama.mwt(x)), args.reps)
    cap = _mwt_grid_cap()

    def mwt_capped():
        with ewvit._lib.grid_cap(cap):
            return dama.mwt(x)
    out['mwt_cap_ms'] = _time(piece(mwt_capped), args.reps)
    out['mwt_cap'] = cap
    out['sfe_ms'] = _time(piece(lambda: dama.sfe(x)), args.reps)
    out['backbone_ms'] = _time(piece(lambda: dama.sfe.efficient_net.features(x)), args.reps)
    from network.losses import combined_loss
    feat = torch.randn(64, 1280, 7, 7, device=dev).to(memory_format=torch.channels_last).requires_grad_(True)
    freq0 = torch.randn(64, 128, 1, 1, device=dev).requires_grad_(True)
    labels = (torch.arange(64, device=dev) % 2).float().view(8, 8)[:, 0]
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([0.5], device=dev))

    xv = torch.zeros(8, 8, 3, 8, 8, device=dev)      # frames are not read: the branches are stubbed

    def tokens():
        # the step's own forward after the two branches (DAMA._process_frame: the fused head
        # when fusable), the classifier and combined_loss, on a fixed backbone map
        dama._branches = lambda frame: (dama.sfe.head(feat).float(), freq0)
        try:
            with torch.autocast('cuda', dtype=torch.bfloat16):
                out_ = model(xv, 8, 'dynamic')
        finally:
            del dama._branches
        return combined_loss(out_, labels, crit, 1, 1)[0]
    out['tokens_ms'] = _time(TrainStep(model, tokens, _NoOpt(model.parameters()), graph=True), args.reps)
    if args.probe_us > 0:
        from network import dama as dm
        cyc = int(args.probe_us * 2100)
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=side):
                torch.cuda._sleep(cyc)
        out['probe_alone_ms'] = _time(g.replay, args.reps)
        orig = dm.BidirectionalCrossTransformer.forward

        def slowed(self, s, f):
            torch.cuda._sleep(cyc)
            return orig(self, s, f)
        dm.BidirectionalCrossTransformer.forward = slowed
        try:
            out['step_probe_ms'] = _time(bench.build_step(dev, 64, 0, graph=True, config=2), args.reps)
        finally:
            dm.BidirectionalCrossTransformer.forward = orig
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
    if args.tables:
        # per-entry event timings of each piece issued eagerly, one stream, uncapped
        pieces = (('mwt', piece(lambda: dama.mwt(x))), ('sfe', piece(lambda: dama.sfe(x))),
                  ('tokens', TrainStep(model, tokens, _NoOpt(model.parameters()), graph=False)))
        for name, st in pieces:
            ewvit._lib.enable_timing(True)
            for _ in range(3):
                st._eager()
            torch.cuda.synchronize()
            tab = bench.kernel_table(ewvit._lib.timing_records())
            shapes = bench.shape_table(ewvit._lib.timing_detail())
            ewvit._lib.enable_timing(False)
            tot = sum(v['total_ms'] for v in tab.values()) / 3
            print(f'--- {name}: {tot:.3f} ms of kernel time per pass, '
                  f'{sum(v["launches"] for v in tab.values()) / 3:.0f} launches')
            for k, v in sorted(tab.items(), key=lambda kv: -kv[1]['total_ms'])[:25]:
                print(f"{k:36s} {v['launches'] / 3:5.0f} {v['total_ms'] / 3:7.3f} ms {v['avg_us']:7.1f} us "
                      f"{v['TFLOP/s']:7.1f} TF/s {v['GB/s']:7.0f} GB/s")
            print(f'top launch configurations ({name}):')
            for r in shapes[:args.tables]:
                print(f"  {r['entry']:34s} {str(r['args'])[:70]:70s} x{r['launches'] / 3:3.0f} "
                      f"{r['total_ms'] / 3:7.3f} ms {r['avg_us']:7.1f} us {r['TFLOP/s']:6.1f} TF/s {r['GB/s']:6.0f} GB/s")


if __name__ == '__main__':
    main()
