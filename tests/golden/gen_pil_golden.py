"""Writes tests/golden/pil_frames.npz: the reference's per-frame transform chain
(config/transforms.py:81-113) computed by Pillow itself — the third-party library the
reference's torchvision Resize / ColorJitter call into — on small synthetic frames.

torchvision is absent here, so its thin layers are the documented ones: Resize(int) size
rule, CenterCrop rounding, ColorJitter -> ImageEnhance.Brightness / Contrast, ToTensor (/255)
and Normalize (float32).  The Pillow parts (the bilinear resample and the blends) are Pillow's
own output.  Run: python tests/golden/gen_pil_golden.py (Pillow 12.2.0).
"""
import os

import numpy as np
import PIL
from PIL import Image, ImageEnhance

MEAN = np.asarray((0.485, 0.456, 0.406), np.float32)[:, None, None]
STD = np.asarray((0.229, 0.224, 0.225), np.float32)[:, None, None]


def frame(rng, h, w):
    """a smooth synthetic frame (compresses well) with a little noise"""
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    base = np.stack([128 + 100 * np.sin(x / (7 + 3 * c) + y / (11 + c)) for c in range(3)], -1)
    return np.clip(base + rng.normal(0, 12, base.shape), 0, 255).astype(np.uint8)


def chain(img, box, size, crop, jitter):
    im = Image.fromarray(img).crop(box)
    w, h = im.size
    short, long = (w, h) if w <= h else (h, w)
    nl = int(size * long / short)
    nw, nh = (size, nl) if w <= h else (nl, size)
    im = im.resize((nw, nh), Image.BILINEAR)
    ox, oy = int(round((nw - crop) / 2.0)), int(round((nh - crop) / 2.0))
    im = im.crop((ox, oy, ox + crop, oy + crop))
    crop_u8 = np.asarray(im)
    if jitter is not None:
        bf, cf, bfirst = jitter
        for op in ('b', 'c') if bfirst else ('c', 'b'):
            im = ImageEnhance.Brightness(im).enhance(bf) if op == 'b' else ImageEnhance.Contrast(im).enhance(cf)
    x = np.asarray(im).transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    return crop_u8, ((x - MEAN) / STD).astype(np.float32)


def main():
    rng = np.random.default_rng(1234)
    cases = [  # (h, w, box or None = centred square, size, crop, jitter)
        (96, 128, None, 80, 48, None),
        (150, 110, (10, 20, 100, 140), 64, 40, (1.007, 0.993, True)),
        (64, 200, (30, 0, 94, 64), 100, 56, (0.991, 1.01, False)),
        (300, 260, None, 96, 64, (1.3, 0.6, True)),          # factors outside [0, 1] clip
        (40, 52, (2, 3, 50, 39), 120, 64, None),               # upscale
    ]
    out = {'pillow_version': np.asarray(PIL.__version__)}
    for i, (h, w, box, size, crop, jit) in enumerate(cases):
        img = frame(rng, h, w)
        if box is None:
            s = min(w, h)
            box = ((w - s) // 2, (h - s) // 2, (w - s) // 2 + s, (h - s) // 2 + s)
        u8, f32 = chain(img, box, size, crop, jit)
        out[f'frame{i}'] = img
        out[f'box{i}'] = np.asarray(box, np.int64)
        out[f'size{i}'] = np.asarray([size, crop], np.int64)
        out[f'jitter{i}'] = np.asarray(jit if jit is not None else (-1.0, -1.0, True), np.float64)
        out[f'crop{i}'] = u8
        out[f'out{i}'] = f32
    out['n'] = np.asarray(len(cases))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'pil_frames.npz')
    np.savez_compressed(path, **out)
    print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
