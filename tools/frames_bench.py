"""Frame transform chain on one MI355X: ewvit_frames_resize_crop over a clip of
64 720p frames with face-sized crop boxes (inputs resident in HBM), timed as back-to-back
launches replayed from one HIP graph, against Pillow + numpy on the host (the reference's own
per-frame CPU path, config/transforms.py:81-113, with torchvision's thin layers restated).

Algorithmic bytes per frame: the source bytes the crop reads (the rows and columns of the box
that reach the 224 x 224 window, 3 B per pixel) + the fp32 output (224*224*3*4 B).

    python tools/frames_bench.py [--frames 64] [--iters 50] [--jitter]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'efficient-wavelet-vit_amd')]

from config.transforms import FrameTransform  # noqa: E402
from oracle import transforms as T  # noqa: E402


def clip(n, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:720, 0:1280]
    base = (128 + 100 * np.sin(x / 9.0 + y / 13.0)).astype(np.uint8)
    frames, boxes = [], []
    for i in range(n):
        f = np.repeat(base[:, :, None], 3, 2)
        f = (f.astype(np.int32) + rng.integers(-20, 20, f.shape)).clip(0, 255).astype(np.uint8)
        s = int(rng.integers(200, 700))
        bx, by = int(rng.integers(0, 1280 - s)), int(rng.integers(0, 720 - s))
        frames.append(f)
        boxes.append((bx, by, bx + s, by + s))
    return frames, boxes


def algorithmic_bytes(boxes, size=450, crop=224):
    tot = 0
    for l, t, r, b in boxes:
        w, h = r - l, b - t
        nw, nh = T.resized_size(w, h, size)
        ox, oy = T.center_crop_offsets(nw, nh, crop)
        hb, _ = T.precompute_coeffs(w, nw)
        vb, _ = T.precompute_coeffs(h, nh)
        cols = hb[ox + crop - 1][0] + hb[ox + crop - 1][1] - hb[ox][0]
        rows = vb[oy + crop - 1][0] + vb[oy + crop - 1][1] - vb[oy][0]
        tot += rows * cols * 3 + crop * crop * 3 * 4
    return tot


def pil_baseline(frames, boxes, budget_s=10.0):
    from PIL import Image
    mean = np.asarray(T.MEAN, np.float32)[:, None, None]
    std = np.asarray(T.STD, np.float32)[:, None, None]
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        f, b = frames[done % len(frames)], boxes[done % len(boxes)]
        im = Image.fromarray(f).crop(b)
        nw, nh = T.resized_size(*im.size)
        im = im.resize((nw, nh), Image.BILINEAR)
        ox, oy = T.center_crop_offsets(nw, nh)
        x = np.asarray(im.crop((ox, oy, ox + 224, oy + 224))).transpose(2, 0, 1).astype(np.float32) / np.float32(255)
        _ = (x - mean) / std
        done += 1
    return done / (time.perf_counter() - t0), done


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=64)
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--jitter', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    args = ap.parse_args()
    from ewvit import _lib
    frames, boxes = clip(args.frames)
    t = FrameTransform(device='cuda', jitter=(0.01, 0.01) if args.jitter else None)
    out = t.batch(frames, boxes)           # warm-up + correctness of one frame
    np.testing.assert_array_equal(out[0].cpu().numpy(), T.transform_frame(frames[0], boxes[0])) \
        if not args.jitter else None
    geom, nbytes = t.geometry(frames, boxes)
    plan = t.plan(geom, nbytes)
    buf = torch.from_numpy(np.concatenate([f.reshape(-1) for f in frames])).cuda()
    g = torch.from_numpy(geom).cuda()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        def launch():
            _lib.call('ewvit_frames_resize_crop', _lib.ptr(buf), _lib.ptr(g), len(frames), 224, plan, 1, t.mean_std,
                      _lib.ptr(out), _lib.stream(out))
        launch()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(args.iters):
                launch()
    with torch.cuda.stream(s):
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        graph.replay()          # replays on the current stream: s
        e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    ab = algorithmic_bytes(boxes)
    # end to end from host frames (pinned copy + geometry + launches), per call
    t0 = time.perf_counter()
    for _ in range(5):
        t.batch(frames, boxes)
    torch.cuda.synchronize()
    e2e_ms = (time.perf_counter() - t0) / 5 * 1e3
    cpu_fps, cpu_n = pil_baseline(frames, boxes, args.cpu_seconds)
    res = {
        'kernel': 'ewvit_frames_resize_crop', 'frames': len(frames), 'plan': list(plan),
        'avg_us': round(us, 2), 'frames_per_s': round(len(frames) / us * 1e6, 1),
        'algorithmic_bytes': ab, 'achieved_GBps': round(ab / us / 1e3, 1), 'peak_GBps': 8000.0,
        'frac': round(ab / us / 1e3 / 8000.0, 4),
        'host_to_output_ms': round(e2e_ms, 3),
        'host_frames_bytes': nbytes,
        'cpu_baseline': {'value': round(cpu_fps, 1), 'unit': 'frames/s', 'cores': 1, 'kind': 'reference',
                         'sample': f'{cpu_n} frames through Pillow crop/resize/crop + numpy normalize '
                                   '(the reference per-frame path, one thread)'},
    }
    print(json.dumps(res))


if __name__ == '__main__':
    main()
