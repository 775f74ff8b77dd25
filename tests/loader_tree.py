"""A synthetic dataset tree in the reference's on-disk layout (config/data_loader.py:76,95,121
for FaceForensics++, :432-433 for Celeb-DF, :608,619 for the diffusion sets), shared by the
fixture generator (tests/golden/gen_loader_golden.py, which runs the reference's loaders on
it) and the CPU parity test (tests/test_data_loader_cpu.py, which runs ours on a fresh copy).

Every frame is a tiny PNG whose pixels are a function of its path, so a clip's pixels pin
which files were selected.  The tree holds the cases the loaders branch on: videos with more
and with fewer frames than frame_count, a video whose frames are .jpg only (the *.png glob is
empty), an unreadable .png (cv2.imread -> None: the blank-frame branch), fake videos available
for 1-3 of the 5 methods, and a Celeb-DF test list with comments, short lines and YouTube rows.
"""
import hashlib
import json
import os

import numpy as np

METHODS = ['Deepfakes', 'Face2Face', 'FaceSwap', 'NeuralTextures', 'FaceShifter']
SPLITS = {'train': 20, 'val': 10, 'test': 10}


def _pixels(rel, hw=(6, 5)):
    seed = int.from_bytes(hashlib.sha1(rel.encode()).digest()[:8], 'little')
    return np.random.default_rng(seed).integers(0, 256, hw + (3,), dtype=np.uint8)


def _write_image(root, rel, ext='.png'):
    from PIL import Image
    path = os.path.join(root, rel)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.fromarray(_pixels(rel)).save(path, format='PNG' if ext == '.png' else 'JPEG', quality=95)


def _video(root, rel_dir, n, ext='.png', corrupt=None):
    for k in range(n):
        rel = os.path.join(rel_dir, f'{k:04d}{ext}')
        if corrupt is not None and k == corrupt:
            path = os.path.join(root, rel)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, 'wb') as f:
                f.write(b'not an image')
        else:
            _write_image(root, rel, ext)


def build(root):
    """Create the tree under `root` (deterministic)."""
    ff = os.path.join(root, 'faceforensics', 'ff++')
    os.makedirs(os.path.join(ff, 'splits'), exist_ok=True)
    vid = 0
    for split, n in SPLITS.items():
        pairs = []
        for _ in range(n):
            t, s = f'{vid:03d}', f'{(vid * 7 + 3) % 100:03d}'
            vid += 1
            pairs.append([t, s])
            nframes = 3 + (vid * 5) % 12              # 3..14 frames
            _video(root, os.path.join('faceforensics', 'ff++', 'frames', 'original', t), nframes,
                   corrupt=2 if vid % 9 == 0 else None)
            for mi, m in enumerate(METHODS):
                if (vid + 2 * mi) % 3 == 0 or (mi == vid % 5):
                    ext = '.jpg' if (vid + mi) % 11 == 0 else '.png'
                    _video(root, os.path.join('faceforensics', 'ff++', 'frames', m, f'{t}_{s}'),
                           2 + (vid + mi) % 13, ext=ext, corrupt=1 if (vid * mi) % 13 == 5 else None)
        with open(os.path.join(ff, 'splits', f'{split}.json'), 'w') as f:
            json.dump(pairs, f)
    cd = os.path.join(root, 'celebdf', 'frames')
    lines = ['// Celeb-DF v2 test list (synthetic)', '']
    for k in range(8):
        _video(root, os.path.join('celebdf', 'frames', 'Celeb-real', f'id{k}_{k:04d}'), 4 + k)
        _video(root, os.path.join('celebdf', 'frames', 'Celeb-synthesis', f'id{k}_id{k + 1}_{k:04d}'), 3 + 2 * k)
        if k % 2 == 0:
            lines.append(f'1 Celeb-real/id{k}_{k:04d}.mp4')
            lines.append(f'0 Celeb-synthesis/id{k}_id{k + 1}_{k:04d}.mp4')
    lines += ['1 YouTube-real/00001.mp4', 'short', '0 Celeb-real/id1_0001.mp4']
    os.makedirs(cd, exist_ok=True)
    with open(os.path.join(root, 'celebdf', 'List_of_testing_videos.txt'), 'w') as f:
        f.write('\n'.join(lines) + '\n')
    dif = os.path.join(root, 'diffusion')
    for k in range(5):
        _write_image(root, os.path.join('diffusion', 'CelebA-Real', f'r{k}.png'))
    for m in ('DDPM', 'DDIM', 'LDM'):
        for k in range(3):
            _write_image(root, os.path.join('diffusion', m, f'{m.lower()}_{k}.png'))
    with open(os.path.join(dif, 'DDPM', 'notes.txt'), 'w') as f:
        f.write('not an image\n')
    return root


def rel(root, p):
    return os.path.relpath(p, root)


def clip_transform(frame):
    """The per-frame transform both sides run in the parity test: the top-left 4 x 4 RGB block
    as a [3, 4, 4] int tensor (blank frames give zeros), so the clip pins the decoded pixels."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(frame[:4, :4])).permute(2, 0, 1).to(torch.int32)


def digest(clip):
    """SHA-1 of a clip tensor's int32 values and shape (what the fixture stores)."""
    import torch
    t = clip.to(torch.int32).contiguous()
    return hashlib.sha1(str(list(t.shape)).encode() + t.numpy().tobytes()).hexdigest()
