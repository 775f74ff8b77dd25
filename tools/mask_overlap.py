"""Experiment: overlap the two DAMA branches by CU-masked streams instead of capped grids.

The MWT branch (forward + backward, uncapped grids) and the SFE branch (backbone + ViT head,
forward + backward) are each captured as their own HIP graph (tools/branch_time.py pieces)
and replayed concurrently, the MWT graph on a stream masked to K CUs and the SFE graph on a
stream masked to the other CUs (or unmasked).  A graph launched on a masked stream runs on
the masked CUs (tools/cumask_probe.py).  Compared with the same pair replayed back to back
and with the capped MWT piece beside the SFE piece on plain streams (today's scheme).

  python tools/mask_overlap.py [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))
sys.path.insert(0, os.path.join(REPO, 'tools'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--prio', action='store_true', help='stream priorities instead of CU masks: the SFE graph '
                    'on a high-priority stream beside the MWT graph on a normal one')
    args = ap.parse_args()
    import bench
    import ewvit
    from branch_time import _NoOpt
    from cumask_probe import masked_stream
    from ewvit.graph import TrainStep
    dev = torch.device('cuda', 0)
    total = torch.cuda.get_device_properties(dev).multi_processor_count
    full = bench.build_step(dev, 64, 0, graph=True, config=2)
    model = full.model
    dama = model.dama
    x = torch.randn(64, 3, 224, 224, device=dev)

    def piece(fn):
        def fl():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                y = fn()
            return y.float().square().mean()
        return TrainStep(model, fl, _NoOpt(model.parameters()), graph=True)

    def capped():
        with ewvit._lib.grid_cap(160):
            return dama.mwt(x)
    st_mwt = piece(lambda: dama.mwt(x))
    st_cap = piece(capped)
    st_sfe = piece(lambda: dama.sfe(x))

    def pair(sa, sb, a, b, reps):
        cur = torch.cuda.current_stream()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        for _ in range(reps):
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            with torch.cuda.stream(sa):
                a()
            with torch.cuda.stream(sb):
                b()
            cur.wait_stream(sa)
            cur.wait_stream(sb)
        e1.record(cur)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    out = {'cus': total}
    plain1, plain2 = torch.cuda.Stream(), torch.cuda.Stream()
    out['serial_ms'] = pair(plain1, plain1, st_mwt, st_sfe, args.reps)
    out['plain_overlap_uncapped_ms'] = pair(plain1, plain2, st_mwt, st_sfe, args.reps)
    out['plain_overlap_cap160_ms'] = pair(plain1, plain2, st_cap, st_sfe, args.reps)
    if args.prio:
        lo, hi = torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)
        out['prio_sfe_hi_uncapped_ms'] = pair(lo, hi, st_mwt, st_sfe, args.reps)
        out['prio_sfe_hi_cap160_ms'] = pair(lo, hi, st_cap, st_sfe, args.reps)
        out['prio_mwt_hi_uncapped_ms'] = pair(hi, lo, st_mwt, st_sfe, args.reps)
        out['plain_overlap_cap160_again_ms'] = pair(plain1, plain2, st_cap, st_sfe, args.reps)
        out['prio_sfe_hi_cap160_again_ms'] = pair(lo, hi, st_cap, st_sfe, args.reps)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
        return
    for k in (96, 128, 160, 192):
        m = masked_stream(k, total)
        # the complement mask for the SFE stream
        import ctypes
        hip = ctypes.CDLL('libamdhip64.so')
        words = (total + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for c in range(k, total):
            mask[c // 32] |= 1 << (c % 32)
        s = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask) == 0
        comp = torch.cuda.ExternalStream(s.value)
        out[f'mask{k}_sfe_complement_ms'] = pair(m, comp, st_mwt, st_sfe, args.reps)
        out[f'mask{k}_sfe_all_ms'] = pair(m, plain2, st_mwt, st_sfe, args.reps)
        out[f'mwt_alone_mask{k}_ms'] = pair(m, m, st_mwt, lambda: None, args.reps)
        out[f'sfe_alone_mask{256 - k}_ms'] = pair(comp, comp, st_sfe, lambda: None, args.reps)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == '__main__':
    main()
