"""GPU parity of the frame transform chain (reference config/transforms.py:81-113
applied per frame by config/data_loader.py:325-337): ewvit_frames_resize_crop /
ewvit_frames_jitter_normalize through config.transforms.FrameTransform against the oracle
(oracle/transforms.py, pinned to Pillow) — bit-exact, uint8 and float32 alike."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import transforms as T


pytestmark = pytest.mark.gpu


def _frames(seed, shapes):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]


SHAPES = [(480, 640), (1080, 1920), (720, 1280), (300, 200), (451, 460), (225, 1000), (2000, 3000), (97, 131)]
BOXES = [None, None, (500, 100, 861, 470), (20, 30, 140, 200), (0, 0, 460, 451), None, (0, 0, 3000, 2000),
         (5, 7, 15, 19)]   # the last: a 10 x 12 box, 45x upscale


def _transform(**kw):
    from config.transforms import FrameTransform
    return FrameTransform(device='cuda', **kw)


def _boxes(frames, boxes):
    return [b if b is not None else T.center_square_box(f.shape[1], f.shape[0]) for f, b in zip(frames, boxes)]


def test_val_batch_bit_exact():
    frames = _frames(0, SHAPES)
    boxes = _boxes(frames, BOXES)
    out = _transform().batch(frames, boxes).cpu().numpy()
    for i, (f, b) in enumerate(zip(frames, boxes)):
        np.testing.assert_array_equal(out[i], T.transform_frame(f, b), err_msg=f'frame {i} {f.shape} {b}')


def test_uint8_image_bit_exact():
    from ewvit import _lib
    frames = _frames(1, SHAPES)
    boxes = _boxes(frames, BOXES)
    t = _transform()
    geom, nbytes = t.geometry(frames, boxes)
    plan = t.plan(geom, nbytes)
    assert 1 <= plan[0] <= 16 and plan[3] > 0      # source rows staged in LDS
    buf = torch.from_numpy(np.concatenate([f.reshape(-1) for f in frames])).cuda()
    g = torch.from_numpy(geom).cuda()
    img = torch.empty(len(frames), 224, 224, 3, dtype=torch.uint8, device='cuda')
    _lib.call('ewvit_frames_resize_crop', _lib.ptr(buf), _lib.ptr(g), len(frames), 224, plan, 0, None,
              _lib.ptr(img), _lib.stream(img))
    img = img.cpu().numpy()
    for i, (f, b) in enumerate(zip(frames, boxes)):
        np.testing.assert_array_equal(img[i], T.resize_center_crop(f, b))
    # one output row per workgroup, and source rows read from global memory (no staging):
    # the same pixels
    for alt in ((1, plan[1], plan[2], plan[3]), (plan[0], plan[1], plan[2], 0)):
        img2 = torch.zeros(len(frames), 224, 224, 3, dtype=torch.uint8, device='cuda')
        _lib.call('ewvit_frames_resize_crop', _lib.ptr(buf), _lib.ptr(g), len(frames), 224, (ctypes.c_int * 4)(*alt),
                  0, None, _lib.ptr(img2), _lib.stream(img2))
        np.testing.assert_array_equal(img2.cpu().numpy(), img, err_msg=str(alt))


def test_train_batch_jitter_bit_exact():
    frames = _frames(2, SHAPES[:6])
    boxes = _boxes(frames, BOXES[:6])
    t = _transform(jitter=(0.01, 0.01))
    torch.manual_seed(7)
    out = t.batch(frames, boxes).cpu().numpy()
    torch.manual_seed(7)
    params = [t._jitter_params() for _ in frames]
    for i, (f, b, (bf, cf, order, _)) in enumerate(zip(frames, boxes, params)):
        ref = T.transform_frame(f, b, jitter=([0, 1] if order == 0 else [1, 0], bf, cf))
        np.testing.assert_array_equal(out[i], ref, err_msg=f'frame {i}')


def test_jitter_wide_factors_bit_exact(monkeypatch):
    """factors outside [0, 1] take Pillow's clipping branch; both orders; one op only"""
    frames = _frames(3, [(300, 400)] * 6)
    boxes = _boxes(frames, [None] * 6)
    params = [[1.6, 0.4, 0.0, 0.0], [0.5, 1.8, 1.0, 0.0], [1.2, -1.0, 0.0, 0.0], [-1.0, 1.3, 0.0, 0.0],
              [0.0, 2.0, 1.0, 0.0], [1.0, 1.0, 0.0, 0.0]]
    it = iter(params)
    t = _transform(jitter=(0.5, 0.5))
    monkeypatch.setattr(t, '_jitter_params', lambda: next(it))
    out = t.batch(frames, boxes).cpu().numpy()
    for i, (f, b, (bf, cf, order, _)) in enumerate(zip(frames, boxes, params)):
        jit = ([0, 1] if order == 0 else [1, 0], bf if bf >= 0 else None, cf if cf >= 0 else None)
        np.testing.assert_array_equal(out[i], T.transform_frame(f, b, jitter=jit), err_msg=f'frame {i}')


def test_pillow_fixture_on_gpu(golden, monkeypatch):
    g = golden('pil_frames.npz')
    for i in range(int(g['n'])):
        size, crop = (int(v) for v in g[f'size{i}'])
        bf, cf, bfirst = g[f'jitter{i}']
        t = _transform(size=size, crop=crop, jitter=None if bf < 0 else (0.5, 0.5))
        monkeypatch.setattr(t, '_jitter_params', lambda: [bf, cf, 0.0 if bfirst else 1.0, 0.0])
        out = t.batch([g[f'frame{i}']], [tuple(int(v) for v in g[f'box{i}'])]).cpu().numpy()[0]
        np.testing.assert_array_equal(out, g[f'out{i}'], err_msg=f'case {i}')


def test_per_frame_call_and_cuda_frames():
    frames = _frames(4, SHAPES[:3])
    t = _transform()
    batch = t.batch(frames)
    for i, f in enumerate(frames):
        torch.testing.assert_close(t(f), batch[i], rtol=0, atol=0)
    dev = t.batch([torch.from_numpy(f).cuda() for f in frames])
    torch.testing.assert_close(dev, batch, rtol=0, atol=0)


def test_full_clip_batch():
    """64 frames of 720p, face-sized boxes: the data path of one BASELINE config-2 step."""
    rng = np.random.default_rng(5)
    frames = _frames(6, [(720, 1280)] * 64)
    boxes = []
    for _ in frames:
        s = int(rng.integers(200, 700))
        x, y = int(rng.integers(0, 1280 - s)), int(rng.integers(0, 720 - s))
        boxes.append((x, y, x + s, y + s))
    t = _transform()
    out = t.batch(frames, boxes)
    again = t.batch(frames, boxes)
    assert torch.equal(out, again)
    out = out.cpu().numpy()
    for i in range(0, 64, 9):
        np.testing.assert_array_equal(out[i], T.transform_frame(frames[i], boxes[i]), err_msg=f'frame {i}')


def test_max_output_size():
    frames = _frames(8, [(600, 800), (1000, 700)])
    t = _transform(size=300, crop=256)
    out = t.batch(frames).cpu().numpy()
    for i, f in enumerate(frames):
        np.testing.assert_array_equal(out[i], T.transform_frame(f, None, size=300, crop=256))


def test_dataset_clip_through_gpu_transform(tmp_path):
    """config/data_loader.py with the GPU transforms (get_transforms()): a FaceForensics++ clip
    is ONE transform.batch launch and equals the reference's per-frame call + torch.stack
    (data_loader.py:333-337) — with the train split's ColorJitter draws in the same order — and
    the oracle (Pillow-pinned) per frame, the blank frame of an unreadable file included."""
    import random
    import loader_tree
    from config import data_loader as D
    from config.transforms import get_transforms
    root = loader_tree.build(str(tmp_path / 'data'))
    tr = get_transforms(device='cuda')
    random.seed(0)
    ds = D.FaceForensicsLoader(root, split='train', frame_count=8, transform=tr['train'])
    for i in (0, 3, len(ds.real_videos) + 1, len(ds) - 1):
        d, _ = ds.video_dir(i)
        frames = D.read_frames(D.select_frames(D.frame_files(d), 8))
        torch.manual_seed(100 + i)
        clip, _ = ds[i]
        torch.manual_seed(100 + i)
        ref = torch.stack([tr['train'](f) for f in frames])
        assert clip.shape == (8, 3, 224, 224) and clip.is_cuda
        assert torch.equal(clip, ref), i
    random.seed(0)
    dv = D.FaceForensicsLoader(root, split='val', frame_count=6, transform=tr['val'])
    blank_seen = False
    for i in range(len(dv)):
        d, _ = dv.video_dir(i)
        frames = D.read_frames(D.select_frames(D.frame_files(d), 6))
        blank_seen |= any(f.shape == (224, 224, 3) and not f.any() for f in frames)
        clip = dv[i][0].cpu().numpy()
        for k, f in enumerate(frames):
            np.testing.assert_array_equal(clip[k], T.transform_frame(f, None), err_msg=f'{i}/{k}')
    assert blank_seen
