"""ORACLE (test infrastructure only) — numpy restatement of the reference's per-frame
transform chain, the input side of the hot path.

Reference call sites:
* ``config/data_loader.py:313``  ``np.linspace(0, len(frame_files) - 1, frame_count, dtype=int)``
  (frame sampling), ``:325-334`` ``cv2.imread`` → BGR2RGB → ``self.transform(frame)`` per
  frame, ``:337`` ``torch.stack``.
* ``config/transforms.py:81-113`` ``get_transforms()``: ToPILImage → FaceAlignTransform(20)
  → Resize(450) → CenterCrop(224) → [ColorJitter(0.01, 0.01), train only] → ToTensor →
  Normalize(ImageNet mean / std).
* ``config/transforms.py:28-79`` ``FaceAlignTransform.__call__``: crop box from the largest
  MTCNN box (``face_box``) or, without a detection, the centred square (``center_square_box``).

Third-party algorithms restated (neither torchvision nor the MTCNN weights are importable
here; Pillow is):
* torchvision ``transforms.Resize(int)`` → ``F._compute_resized_output_size`` (short side =
  size, long side = ``int(size * long / short)``) → ``PIL.Image.resize(.., BILINEAR)``.
* Pillow ``Resample.c`` (``ImagingResampleInner``): separable bilinear with support
  ``max(scale, 1)``; coefficients in double, normalised per output sample, then fixed point
  with ``PRECISION_BITS = 22`` (round half away from zero); the horizontal pass runs first
  over the rows the vertical pass needs, each pass rounds ``(acc + 2^21) >> 22`` and clips to
  uint8.
* torchvision ``CenterCrop`` → ``crop_top = int(round((h - 224) / 2.0))`` (Python rounding).
* torchvision ``ColorJitter`` on PIL: ``ImageEnhance.Brightness`` = ``Image.blend(black,
  img, f)``; ``ImageEnhance.Contrast`` = blend with the grey image of
  ``int(mean(img.convert('L')) + 0.5)``, ``L = (19595 R + 38470 G + 7471 B + 0x8000) >> 16``;
  ``ImagingBlend``: ``float`` arithmetic ``in1 + alpha * (in2 - in1)``, truncated to uint8
  inside [0, 1], clipped outside.
* ``ToTensor`` (``/ 255`` in float32) and ``Normalize`` (``(x - mean) / std`` in float32).

Pinned against Pillow 12.2.0 itself (``tests/test_transforms_cpu.py`` runs both on random
frames, sizes and boxes) and by ``tests/golden/pil_frames.npz`` (``gen_pil_golden.py``).
"""
import numpy as np

PRECISION_BITS = 22
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def sample_frame_indices(n_files, frame_count):
    """``config/data_loader.py:313``."""
    return np.linspace(0, n_files - 1, frame_count, dtype=int).tolist()


def center_square_box(w, h):
    """``config/transforms.py:72-79`` (no face found): the centred square."""
    s = min(w, h)
    left, top = (w - s) // 2, (h - s) // 2
    return left, top, left + s, top + s


def face_box(box, margin, w, h):
    """``config/transforms.py:52-67``: crop around an MTCNN box ``(x0, y0, x1, y1)``."""
    cx, cy = (box[0] + box[2]) / 2, (box[1] + box[3]) / 2
    fs = max(box[2] - box[0], box[3] - box[1])
    cs = fs + margin * 2
    return (int(max(0, cx - cs / 2)), int(max(0, cy - cs / 2)),
            int(min(w, cx + cs / 2)), int(min(h, cy + cs / 2)))


def resized_size(w, h, size=450):
    """torchvision ``_compute_resized_output_size`` for ``Resize(int)`` -> (new_w, new_h)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_short, new_long) if w <= h else (new_long, new_short)


def center_crop_offsets(w, h, crop=224):
    """torchvision ``F.center_crop`` on a PIL image -> (left, top)."""
    return int(round((w - crop) / 2.0)), int(round((h - crop) / 2.0))


def precompute_coeffs(in_size, out_size):
    """Pillow ``precompute_coeffs`` (box = whole input) + ``normalize_coeffs_8bpc``:
    per output sample (xmin, n) and n int32 weights."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ss = 1.0 / filterscale
    bounds, coeffs = [], []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            k.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum_seq(k)
        if ww != 0.0:
            k = [v / ww for v in k]
        kk = [int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
              for v in k]
        bounds.append((xmin, xmax))
        coeffs.append(kk)
    return bounds, coeffs


def sum_seq(vals):
    s = 0.0
    for v in vals:
        s += v
    return s


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resample_axis(img, axis, bounds, coeffs, out_idx):
    """One 8-bpc pass of ``ImagingResampleHorizontal/Vertical_8bpc`` over ``axis`` of an
    HWC uint8 image, for the output samples ``out_idx`` only."""
    img = np.moveaxis(img.astype(np.int64), axis, 0)
    out = np.empty((len(out_idx),) + img.shape[1:], np.uint8)
    for o, xx in enumerate(out_idx):
        xmin, n = bounds[xx]
        acc = np.full(img.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for x in range(n):
            acc += img[xmin + x] * coeffs[xx][x]
        out[o] = _clip8(acc)
    return np.moveaxis(out, 0, axis)


def resize_center_crop(frame, box, size=450, crop=224):
    """uint8 HWC frame -> crop ``box`` -> Resize(size) -> CenterCrop(crop) (uint8 HWC),
    computing only the pixels the crop keeps (Pillow computes them the same way: each pass
    is independent per output row / column)."""
    l, t, r, b = box
    src = frame[t:b, l:r]
    h, w = src.shape[:2]
    nw, nh = resized_size(w, h, size)
    ox, oy = center_crop_offsets(nw, nh, crop)
    hb, hc = precompute_coeffs(w, nw)
    vb, vc = precompute_coeffs(h, nh)
    rows = range(oy, oy + crop)
    y0 = min(vb[y][0] for y in rows)
    y1 = max(vb[y][0] + vb[y][1] for y in rows)
    need_h = nw != w
    need_v = nh != h
    tmp = resample_axis(src[y0:y1], 1, hb, hc, range(ox, ox + crop)) if need_h else src[y0:y1, ox:ox + crop]
    vb = [(a - y0, n) for a, n in vb]
    return resample_axis(tmp, 0, vb, vc, rows) if need_v else tmp[oy - y0:oy - y0 + crop]


def blend(img1, img2, alpha):
    """Pillow ``ImagingBlend`` (uint8, float32 arithmetic)."""
    a = np.float32(alpha)
    i1, i2 = img1.astype(np.float32), img2.astype(np.float32)
    v = (i1 + a * (i2 - i1)).astype(np.float32)
    return np.clip(np.trunc(v), 0, 255).astype(np.uint8)


def luma_mean_level(img):
    """``int(ImageStat.Stat(img.convert('L')).mean[0] + 0.5)``."""
    x = img.astype(np.int64)
    L = (x[..., 0] * 19595 + x[..., 1] * 38470 + x[..., 2] * 7471 + 0x8000) >> 16
    return int(L.sum() / L.size + 0.5)


def adjust_brightness(img, f):
    return blend(np.zeros_like(img), img, f)


def adjust_contrast(img, f):
    return blend(np.full_like(img, luma_mean_level(img)), img, f)


def color_jitter(img, order, brightness, contrast):
    """torchvision ``ColorJitter.forward`` with saturation / hue unset: ``order`` is
    ``torch.randperm(4)``; ids 0 / 1 are brightness / contrast, 2 / 3 are no-ops."""
    for fn in order:
        if fn == 0 and brightness is not None:
            img = adjust_brightness(img, brightness)
        elif fn == 1 and contrast is not None:
            img = adjust_contrast(img, contrast)
    return img


def to_tensor_normalize(img, mean=MEAN, std=STD):
    """``ToTensor`` + ``Normalize``: uint8 HWC -> float32 CHW."""
    x = np.ascontiguousarray(img.transpose(2, 0, 1)).astype(np.float32) / np.float32(255)
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    return ((x - m) / s).astype(np.float32)


def transform_frame(frame, box=None, jitter=None, size=450, crop=224):
    """The whole chain for one HWC uint8 RGB frame.  ``box`` defaults to the centred
    square (no face detected); ``jitter`` = (order, brightness, contrast) or None (val /
    test transform)."""
    h, w = frame.shape[:2]
    box = box if box is not None else center_square_box(w, h)
    img = resize_center_crop(frame, box, size, crop)
    if jitter is not None:
        img = color_jitter(img, *jitter)
    return to_tensor_normalize(img)
