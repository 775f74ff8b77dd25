"""The reference's frame transforms (config/transforms.py) on the MI355X.

Reference: ``config/transforms.py:81-113`` ``get_transforms()`` builds, per split,
``ToPILImage -> FaceAlignTransform(margin=20) -> Resize(450) -> CenterCrop(224) ->
[ColorJitter(brightness=0.01, contrast=0.01), train only] -> ToTensor -> Normalize(ImageNet)``,
and the datasets call it once per frame before stacking (``config/data_loader.py:325-337``).

Here ``get_transforms()`` returns the same three pipelines as :class:`FrameTransform` objects:

* ``t(frame)`` — the reference's per-frame call: an HWC uint8 RGB frame in, ``[3, 224, 224]``
  float32 out (on the GPU);
* ``t.batch(frames)`` — all frames of a clip (ragged sizes) in one host->device copy and one
  ``ewvit_frames_resize_crop`` launch (plus ``ewvit_frames_jitter_normalize`` for the train
  split): ``[N, 3, 224, 224]``, bit-identical to stacking the per-frame outputs of Pillow +
  torchvision (tests/test_gpu_frames.py against oracle/transforms.py, itself pinned to Pillow).

The face box: ``FaceAlignTransform`` keeps the reference's crop arithmetic
(``transforms.py:52-79``).  MTCNN (facenet_pytorch and its weights) is not available offline, so
the detector is a constructor argument — any callable ``frame -> boxes [k, 4]`` or ``None``;
without one, or when it finds no face, the crop is the reference's fallback (the centred square).

There is no CPU path: the kernels run on the GPU only (``ewvit._lib`` raises without the library).
"""
import ctypes

import numpy as np
import torch

from ewvit import _lib

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def sample_frame_indices(n_files, frame_count):
    """The frames a clip uses (``config/data_loader.py:313``)."""
    return np.linspace(0, n_files - 1, frame_count, dtype=int).tolist()


def resized_size(w, h, size):
    """torchvision ``Resize(int)``: the short side becomes ``size``, the long side
    ``int(size * long / short)`` -> (new_w, new_h)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_short, new_long) if w <= h else (new_long, new_short)


def center_crop_offsets(w, h, crop):
    """torchvision ``CenterCrop`` on a PIL image -> (left, top)."""
    return int(round((w - crop) / 2.0)), int(round((h - crop) / 2.0))


class FaceAlignTransform:
    """``config/transforms.py:14-79``: the crop box of a frame (the crop itself is done by the
    resize kernel, which reads the box straight out of the frame)."""

    def __init__(self, margin, detector=None):
        self.margin = margin
        self.detector = detector

    def box(self, frame):
        h, w = frame.shape[:2]
        boxes = None
        if self.detector is not None:
            try:
                boxes = self.detector(frame)
            except Exception as e:        # transforms.py:68-69
                print(f"Failed to detect face: {e}")
                boxes = None
        if boxes is not None and len(boxes) > 0:
            box = sorted(boxes, key=lambda x: (x[2] - x[0]) * (x[3] - x[1]), reverse=True)[0]
            cx, cy = (box[0] + box[2]) / 2, (box[1] + box[3]) / 2
            fs = max(box[2] - box[0], box[3] - box[1])
            cs = fs + self.margin * 2
            return (int(max(0, cx - cs / 2)), int(max(0, cy - cs / 2)),
                    int(min(w, cx + cs / 2)), int(min(h, cy + cs / 2)))
        s = min(w, h)                     # transforms.py:72-79: the centred square
        left, top = (w - s) // 2, (h - s) // 2
        return left, top, left + s, top + s


class FrameTransform:
    """One pipeline of ``get_transforms()``: crop box -> Resize(size) -> CenterCrop(crop) ->
    [ColorJitter(brightness, contrast)] -> ToTensor -> Normalize(mean, std)."""

    def __init__(self, jitter=None, size=450, crop=224, margin=20, mean=MEAN, std=STD, detector=None,
                 device=None):
        self.face = FaceAlignTransform(margin, detector)
        self.jitter = jitter              # (brightness, contrast) ranges as ColorJitter's, or None
        self.size, self.crop = int(size), int(crop)
        self.mean_std = (ctypes.c_float * 6)(*[float(v) for v in tuple(mean) + tuple(std)])
        self.device = torch.device(device) if device is not None else None

    # torchvision ColorJitter.get_params with saturation / hue unset: the order of the four
    # adjustments, then one factor per set range (uniform in [max(0, 1 - j), 1 + j])
    def _jitter_params(self):
        b, c = self.jitter
        order = torch.randperm(4).tolist()
        bf = float(torch.empty(1).uniform_(max(0.0, 1 - b), 1 + b)) if b else -1.0
        cf = float(torch.empty(1).uniform_(max(0.0, 1 - c), 1 + c)) if c else -1.0
        return [bf, cf, 0.0 if order.index(0) < order.index(1) else 1.0, 0.0]

    def geometry(self, frames, boxes=None):
        """[n][10] int64 (include/ewvit.h ewvit_frames_plan) and the total bytes."""
        geom, off = [], 0
        for i, f in enumerate(frames):
            h, w = int(f.shape[0]), int(f.shape[1])
            if f.ndim != 3 or f.shape[2] != 3:
                raise ValueError(f'frame {i}: expected HWC RGB, got shape {tuple(f.shape)}')
            l, t, r, b = boxes[i] if boxes is not None else self.face.box(f)
            cw, ch = r - l, b - t
            nw, nh = resized_size(cw, ch, self.size)
            ox, oy = center_crop_offsets(nw, nh, self.crop)
            geom.append([off, 3 * w, l, t, cw, ch, nw, nh, ox, oy])
            off += h * w * 3
        return np.asarray(geom, np.int64).reshape(-1, 10), off

    def plan(self, geom, nbytes):
        """ewvit_frames_plan: validate the geometry on the host, the launch shape (int[4])."""
        lib = _lib.load()
        plan = (ctypes.c_int * 4)()
        if lib.ewvit_frames_plan(geom.ctypes.data_as(ctypes.c_void_p), len(geom), self.crop, nbytes, plan):
            raise ValueError(f'ewvit_frames_plan: {lib.ewvit_last_error().decode()}')
        return plan

    def batch(self, frames, boxes=None):
        """frames: sequence of HWC uint8 RGB arrays / tensors (any sizes) -> [N, 3, crop, crop]."""
        frames = [f if isinstance(f, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(f)) for f in frames]
        if not frames:
            raise ValueError('FrameTransform.batch: no frames')
        for f in frames:
            if f.dtype != torch.uint8:
                raise TypeError(f'frames must be uint8 (cv2.imread output), got {f.dtype}')
        dev = self.device or (frames[0].device if frames[0].is_cuda else torch.device('cuda'))
        geom, nbytes = self.geometry(frames, boxes)
        n, S = len(frames), self.crop
        plan = self.plan(geom, nbytes)
        if all(f.is_cuda for f in frames):
            buf = torch.cat([f.reshape(-1) for f in frames])
        else:
            host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            off = 0
            for f in frames:
                k = f.numel()
                host[off:off + k].copy_(f.reshape(-1))
                off += k
            buf = host.to(dev, non_blocking=True)
        g = torch.from_numpy(geom).pin_memory().to(dev, non_blocking=True)
        out = torch.empty(n, 3, S, S, dtype=torch.float32, device=dev)
        _lib.require_gpu(buf, out)
        with torch.cuda.device(dev):
            stream = _lib.stream(out)
            if self.jitter is None:
                _lib.call('ewvit_frames_resize_crop', _lib.ptr(buf), _lib.ptr(g), n, S, plan, 1, self.mean_std,
                          _lib.ptr(out), stream)
            else:
                img = torch.empty(n, S, S, 3, dtype=torch.uint8, device=dev)
                jit = torch.tensor([self._jitter_params() for _ in range(n)], dtype=torch.float32)
                jit = jit.pin_memory().to(dev, non_blocking=True)
                _lib.call('ewvit_frames_resize_crop', _lib.ptr(buf), _lib.ptr(g), n, S, plan, 0, None,
                          _lib.ptr(img), stream)
                _lib.call('ewvit_frames_jitter_normalize', _lib.ptr(img), _lib.ptr(jit), n, S, self.mean_std,
                          _lib.ptr(out), stream)
        return out

    def __call__(self, frame):
        """The reference's per-frame call (``data_loader.py:334``): [3, crop, crop]."""
        return self.batch([frame])[0]


def get_transforms(detector=None, device=None):
    """``config/transforms.py:81-113``: {'train', 'val', 'test'} pipelines."""
    return {
        'train': FrameTransform(jitter=(0.01, 0.01), detector=detector, device=device),
        'val': FrameTransform(detector=detector, device=device),
        'test': FrameTransform(detector=detector, device=device),
    }
