"""CPU checks of the frame transform chain (reference config/transforms.py:81-113):
the oracle restatement against Pillow itself (random frames, boxes and scales) and against the
committed Pillow fixture, the host-side geometry of the product (crop box, Resize size,
CenterCrop offsets) against the oracle, and the C-ABI planner's validation (host-only, no GPU)."""
import ctypes

import numpy as np
import pytest

from oracle import transforms as T

PIL = pytest.importorskip('PIL')
from PIL import Image, ImageEnhance  # noqa: E402


def _pil_chain(frame, box, size=450, crop=224):
    im = Image.fromarray(frame).crop(box)
    nw, nh = T.resized_size(*im.size, size)
    im = im.resize((nw, nh), Image.BILINEAR)
    ox, oy = T.center_crop_offsets(nw, nh, crop)
    return np.asarray(im.crop((ox, oy, ox + crop, oy + crop)))


CASES = [  # (h, w, box or None)
    (480, 640, None),                     # centred square, 480 -> 450
    (1080, 1920, None),                   # 1080 -> 450 (2.4x down, 7 taps)
    (720, 1280, (500, 100, 861, 470)),    # a face-sized box, ~0.8x
    (300, 200, (20, 30, 140, 200)),       # small box, upscale 3.75x
    (2000, 3000, (0, 0, 3000, 2000)),     # 4.4x down, non-square
    (460, 451, (0, 0, 451, 460)),         # almost 1:1
    (225, 1000, None),                    # square of 225 -> 450 (exactly 2x up)
]


@pytest.mark.parametrize('h,w,box', CASES)
def test_oracle_resize_matches_pillow(h, w, box):
    rng = np.random.default_rng(h * 7 + w)
    frame = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    box = box or T.center_square_box(w, h)
    np.testing.assert_array_equal(T.resize_center_crop(frame, box), _pil_chain(frame, box))


def test_oracle_resize_random_pillow():
    rng = np.random.default_rng(0)
    for _ in range(40):
        h, w = int(rng.integers(100, 600)), int(rng.integers(100, 600))
        frame = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        x0, y0 = int(rng.integers(0, w - 50)), int(rng.integers(0, h - 50))
        box = (x0, y0, int(rng.integers(x0 + 40, w + 1)), int(rng.integers(y0 + 40, h + 1)))
        size, crop = int(rng.integers(60, 300)), int(rng.integers(16, 60))
        np.testing.assert_array_equal(T.resize_center_crop(frame, box, size, crop),
                                      _pil_chain(frame, box, size, crop))


def test_oracle_jitter_matches_pillow():
    rng = np.random.default_rng(1)
    for _ in range(30):
        img = rng.integers(0, 256, (50, 60, 3), dtype=np.uint8)
        b, c = float(rng.uniform(0.3, 1.7)), float(rng.uniform(0.3, 1.7))
        p = Image.fromarray(img)
        np.testing.assert_array_equal(T.adjust_brightness(img, b), np.asarray(ImageEnhance.Brightness(p).enhance(b)))
        np.testing.assert_array_equal(T.adjust_contrast(img, c), np.asarray(ImageEnhance.Contrast(p).enhance(c)))
        assert T.luma_mean_level(img) == int(np.asarray(p.convert('L')).mean() + 0.5)


def test_oracle_against_pillow_fixture(golden):
    g = golden('pil_frames.npz')
    for i in range(int(g['n'])):
        size, crop = (int(v) for v in g[f'size{i}'])
        bf, cf, bfirst = g[f'jitter{i}']
        u8 = T.resize_center_crop(g[f'frame{i}'], tuple(int(v) for v in g[f'box{i}']), size, crop)
        np.testing.assert_array_equal(u8, g[f'crop{i}'])
        jit = None if bf < 0 else ([0, 1] if bfirst else [1, 0], bf, cf)
        img = T.color_jitter(u8, *jit) if jit else u8
        np.testing.assert_array_equal(T.to_tensor_normalize(img), g[f'out{i}'])


def test_frame_indices_and_face_box():
    assert T.sample_frame_indices(100, 8) == np.linspace(0, 99, 8, dtype=int).tolist()
    assert T.sample_frame_indices(5, 8) == [0, 0, 1, 1, 2, 2, 3, 4]
    assert T.face_box((100.0, 120.0, 180.0, 220.0), 20, 640, 480) == (70, 100, 210, 240)
    assert T.face_box((0.0, 0.0, 50.0, 60.0), 20, 640, 480) == (0, 0, 75, 80)


def test_product_geometry_matches_oracle():
    from config.transforms import FaceAlignTransform, FrameTransform
    rng = np.random.default_rng(2)
    frames = [np.zeros((int(rng.integers(100, 900)), int(rng.integers(100, 900)), 3), np.uint8) for _ in range(12)]
    boxes = [None] * 6 + [[(30.0, 40.0, 90.0, 120.0)]] * 6
    det = iter(boxes)
    t = FrameTransform(detector=lambda f: next(det))
    geom, nbytes = t.geometry(frames)
    assert nbytes == sum(f.size for f in frames)
    off = 0
    for f, g, b in zip(frames, geom, boxes):
        h, w = f.shape[:2]
        box = T.center_square_box(w, h) if b is None else T.face_box(b[0], 20, w, h)
        nw, nh = T.resized_size(box[2] - box[0], box[3] - box[1])
        ox, oy = T.center_crop_offsets(nw, nh)
        assert list(g) == [off, 3 * w, box[0], box[1], box[2] - box[0], box[3] - box[1], nw, nh, ox, oy]
        off += f.size
    assert FaceAlignTransform(20).box(frames[0]) == T.center_square_box(frames[0].shape[1], frames[0].shape[0])


def test_planner_validates_on_the_host():
    """ewvit_frames_plan runs on the host: launch shape and argument checks, no GPU."""
    from config.transforms import FrameTransform
    from ewvit import _lib
    lib = _lib.load()

    def plan(frames, nbytes=None, S=224):
        t = FrameTransform(crop=S)
        geom, nb = t.geometry(frames)
        out = (ctypes.c_int * 4)()
        rc = lib.ewvit_frames_plan(geom.ctypes.data_as(ctypes.c_void_p), len(frames), S,
                                   nb if nbytes is None else nbytes, out)
        return rc, list(out)

    rc, p = plan([np.zeros((480, 640, 3), np.uint8)])
    assert rc == 0 and p[0] == 4 and p[1] == 5 and p[3] > 0            # staged; 480 -> 450: support 2
    rc, p = plan([np.zeros((1080, 1920, 3), np.uint8), np.zeros((2000, 3000, 3), np.uint8)])
    assert rc == 0 and 1 <= p[0] < 16 and p[1] == 2 * 5 + 1             # 4.4x down: 11 taps
    rc, _ = plan([np.zeros((480, 640, 3), np.uint8)], nbytes=1000)
    assert rc != 0 and b'bad geometry' in lib.ewvit_last_error()
    rc, _ = plan([np.zeros((4000, 4000, 3), np.uint8)])
    assert rc != 0 and b'beyond 8x' in lib.ewvit_last_error()
    rc, _ = plan([np.zeros((480, 640, 3), np.uint8)], S=300)
    assert rc != 0
