"""The reference's datasets (config/data_loader.py) — the host half of SURVEY §8 row N4.

Same classes, constructor arguments, attributes and sampling behaviour as the reference:

* ``FaceForensicsLoader`` (data_loader.py:10-339): the FF++ split walk, one fake video per
  target/source pair picked from the least-used method, and the training curriculum —
  a fixed fake subset early, a usage-ordered "novel" pool mixed in from 30 % to 70 % of the
  epochs (``update_sampling_strategy``, called by train.py:290-291 every epoch); the val split
  keeps 80 % of the fakes fixed and redraws the other 20 % per epoch.  All draws go through
  Python's global ``random`` in the reference's order, so a seeded run picks the same videos;
* ``CelebDFLoader`` (:342-538) and ``DiffusionLoader`` (:540-711), used by eval.py.

``__getitem__`` assembles a clip as the reference does (:305-339): the sorted frame files,
``np.linspace`` selection when there are more than ``frame_count``, the last frame repeated
when there are fewer, a blank 224 × 224 frame for a file that does not decode, then the
transform.  With a ``config.transforms.FrameTransform`` (``get_transforms()``) the whole clip
goes through ONE ``transform.batch(frames)`` — one host->device copy of the raw frames and one
``ewvit_frames_resize_crop`` launch — bit-identical to the reference's per-frame call +
``torch.stack``; any other callable is applied per frame as in the reference.

Decoding: ``cv2.imread`` + ``cvtColor(BGR2RGB)`` when OpenCV is importable (as the reference);
otherwise Pillow, converted to 8-bit RGB with the EXIF orientation applied (what
``cv2.imread``'s IMREAD_COLOR does).  For PNG frames (lossless) both give the same pixels; for
JPEG the two libraries' IDCTs may differ by a unit in some pixels — JPEG decode parity is
unpinned (tests/test_data_loader_cpu.py pins everything else against the reference's own
loaders, tests/golden/ref_loader.json).

The GPU transform runs in the calling process: keep ``num_workers=0`` (as train.py:226 does), or
load raw clips in the workers (``transform=None``-style callables) and call
``transform.batch`` on the main process.
"""
import glob
import json
import os
import random

import numpy as np
import torch
from torch.utils.data import Dataset

BLANK_HW = 224            # the placeholder frame for an unreadable file (data_loader.py:330)
FF_METHODS = ['Deepfakes', 'Face2Face', 'FaceSwap', 'NeuralTextures', 'FaceShifter']

try:                      # pragma: no cover - OpenCV is not part of this image
    import cv2 as _cv2
except ImportError:       # pragma: no cover
    _cv2 = None


def imread_rgb(path):
    """An HWC uint8 RGB frame, or None when the file cannot be read (cv2.imread's contract)."""
    if _cv2 is not None:
        img = _cv2.imread(path)
        return None if img is None else _cv2.cvtColor(img, _cv2.COLOR_BGR2RGB)
    from PIL import Image, ImageOps
    try:
        with Image.open(path) as im:
            im = ImageOps.exif_transpose(im)
            return np.array(im.convert("RGB"))
    except Exception:     # noqa: BLE001 — unreadable / not an image: the caller's blank frame
        return None


def frame_files(frames_dir, jpg_fallback=True):
    """Sorted *.png of a video directory, else (FF++ only) its *.jpg (data_loader.py:306-308)."""
    files = sorted(glob.glob(os.path.join(frames_dir, '*.png')))
    if not files and jpg_fallback:
        files = sorted(glob.glob(os.path.join(frames_dir, '*.jpg')))
    return files


def select_frames(files, frame_count):
    """``frame_count`` files: evenly spaced when there are more (np.linspace, truncated to
    int), else all of them with the last one repeated (data_loader.py:311-320; an empty list
    raises IndexError, as the reference's padding loop does)."""
    if len(files) > frame_count:
        return [files[i] for i in np.linspace(0, len(files) - 1, frame_count, dtype=int).tolist()]
    out = list(files)
    while len(out) < frame_count:
        out.append(files[-1])
    return out


def read_frames(paths, imread=None):
    """Decoded RGB frames; a blank BLANK_HW² frame stands in for each unreadable file."""
    imread = imread or imread_rgb
    frames = []
    for p in paths:
        img = imread(p)
        frames.append(img if img is not None else np.zeros((BLANK_HW, BLANK_HW, 3), dtype=np.uint8))
    return frames


def apply_transform(frames, transform):
    """The clip tensor [T, C, H, W]: one batched launch for an ewvit FrameTransform, else the
    reference's per-frame call and stack of the tensor results (data_loader.py:333-337)."""
    if transform is not None and hasattr(transform, 'batch') and frames:
        return transform.batch(frames)
    if transform:
        frames = [transform(f) for f in frames]
    return torch.stack([f for f in frames if isinstance(f, torch.Tensor)])


class _ClipDataset(Dataset):
    """Clip assembly shared by the video datasets."""

    _jpg_fallback = True
    imread = staticmethod(imread_rgb)

    def _clip(self, frames_dir):
        files = frame_files(frames_dir, self._jpg_fallback)
        if not files and not self._jpg_fallback:
            raise FileNotFoundError(f"No frames found in '{frames_dir}'")
        return apply_transform(read_frames(select_frames(files, self.frame_count), type(self).imread),
                               self.transform)


# ------------------------------------------------------------------ FaceForensics++
def _fake_candidates(root, methods, video_ids):
    """{target_source: [candidate videos in method order]} (data_loader.py:118-137)."""
    by_pair = {}
    for method in methods:
        mdir = os.path.join(root, 'faceforensics/ff++/frames', method)
        if not os.path.exists(mdir):
            raise FileNotFoundError(f"Fake videos directory '{mdir}' not found")
        for target, source in video_ids:
            d = os.path.join(mdir, f'{target}_{source}')
            if os.path.exists(d):
                by_pair.setdefault(f'{target}_{source}', []).append(
                    {'path': d, 'method': method, 'target': target, 'source': source})
    return by_pair


def _balanced_pick(by_pair, methods):
    """One fake per pair, from the method picked least so far; ties keep method order
    (a stable sort, data_loader.py:147-155)."""
    used = dict.fromkeys(methods, 0)
    picked = []
    for cands in by_pair.values():
        cands.sort(key=lambda v: used[v['method']])
        picked.append(cands[0])
        used[cands[0]['method']] += 1
    return picked


def curriculum_ratios(epoch, max_epochs, early=0.3, late=0.7):
    """(fixed_sample_ratio, novelty_ratio) of a training epoch (data_loader.py:240-260): all
    fixed before ``early`` of the run, then a linear hand-over reaching all-novel at ``late``."""
    if epoch < max_epochs * early:
        return 1.0, 0.0
    progress = min(1.0, (epoch - max_epochs * early) / (max_epochs * (late - early)))
    return max(0.0, 1.0 - progress), min(1.0, progress)


class FaceForensicsLoader(_ClipDataset):
    """FaceForensics++ clips (reference config/data_loader.py:10-339)."""

    def __init__(self, root, split='train', frame_count=24, transform=None, compression='C23',
                 methods=FF_METHODS, fixed_sample_ratio=1.0, novelty_ratio=0.0, single_method=None):
        super().__init__()
        self.root, self.split, self.frame_count, self.transform = root, split, frame_count, transform
        self.compression, self.methods, self.single_method = compression, methods, single_method
        self.fixed_sample_ratio, self.novelty_ratio = fixed_sample_ratio, novelty_ratio
        self.current_epoch = 0
        self.split_ids = self._load_split()
        self.all_fake_videos_by_method = {}
        self.video_usage_counts = {}
        self.real_videos, self.fake_videos = self._load_frames_dirs(self.methods)
        self._init_sampling_strategy()
        print(f'Loaded {len(self.real_videos)} real videos and {len(self.fake_videos)} fake videos')

    def __len__(self):
        fakes = self.current_fake if self.split in ('train', 'val') else self.fake_videos
        return len(self.real_videos) + len(fakes)

    def _load_split(self):
        path = os.path.join(self.root, f'faceforensics/ff++/splits/{self.split}.json')
        if not os.path.exists(path):
            raise FileNotFoundError(f"Split file '{path}' not found")
        with open(path) as f:
            return json.load(f)

    def _load_frames_dirs(self, methods):
        """(real video dirs, fake video records) of the split, data_loader.py:83-169."""
        orig = os.path.join(self.root, 'faceforensics/ff++/frames/original')
        if not os.path.exists(orig):
            raise FileNotFoundError(f"Original video frames directory '{orig}' not found")
        video_ids = list(self.split_ids)
        real = [os.path.join(orig, f'{pair[0]}') for pair in video_ids]
        for d in real:
            if not os.path.exists(d):
                raise Exception(f"Original video '{d}' not found")   # noqa: TRY002 — the reference's type
        if len(real) // len(self.methods) <= 0:
            raise ValueError(f'Invalid number of samples per method: {len(real) // len(self.methods)}')
        by_pair = _fake_candidates(self.root, self.methods, video_ids)
        if self.split == 'test' and self.single_method is not None:
            fake = [v for cands in by_pair.values() for v in cands if v['method'] == self.single_method]
        else:
            fake = _balanced_pick(by_pair, self.methods)
        random.shuffle(fake)              # mixes the methods; the first global-`random` draw
        counts = {}
        for v in fake:
            counts[v['method']] = counts.get(v['method'], 0) + 1
        print('Selected videos by method:')
        for m, c in counts.items():
            print(f'  - {m}: {c} videos')
        return real, fake

    def _init_sampling_strategy(self):
        """The epoch-0 fake subsets (data_loader.py:171-194)."""
        self.video_usage_counts.update((v['path'], 0) for v in self.fake_videos)
        n = len(self.fake_videos)
        if self.split == 'train':
            self.fixed_fake = random.sample(self.fake_videos, int(n * self.fixed_sample_ratio))
            self.pool_fake = [v for v in self.fake_videos if v not in self.fixed_fake]
            self.current_fake = list(self.fixed_fake)
        elif self.split == 'val':
            random.seed(42)
            self.core_fake = random.sample(self.fake_videos, int(n * 0.8))
            self.dynamic_pool_fake = [v for v in self.fake_videos if v not in self.core_fake]
            random.seed(42)
            self.dynamic_fake = self._draw_dynamic()
            self.current_fake = self.core_fake + self.dynamic_fake

    def _draw_dynamic(self):
        return random.sample(self.dynamic_pool_fake, min(int(len(self.fake_videos) * 0.2), len(self.dynamic_pool_fake)))

    def _refresh_training_samples(self):
        """Re-draw the training fakes for the current ratios (data_loader.py:196-227): a random
        part of the fixed set, the least-used pool videos, random other pool videos."""
        n = len(self.fake_videos)
        n_fixed = int(n * self.fixed_sample_ratio)
        kept = random.sample(self.fixed_fake, n_fixed) if n_fixed > 0 else []
        rest = n - n_fixed
        self.pool_fake.sort(key=lambda v: self.video_usage_counts[v['path']])   # stable, persists
        n_new = int(rest * self.novelty_ratio)
        n_rand = rest - n_new
        tail = self.pool_fake[n_new:]
        drawn = random.sample(tail, min(n_rand, len(tail))) if (n_rand > 0 and tail) else []
        merged = {}
        for v in kept + self.pool_fake[:n_new] + drawn:
            merged[v['path']] = v        # first position, last record (no duplicates)
        self.current_fake = list(merged.values())
        random.shuffle(self.current_fake)

    def update_sampling_strategy(self, epoch, max_epochs):
        """Called once per epoch by train.py:290-291 (data_loader.py:229-268)."""
        self.current_epoch = epoch
        if self.split == 'train':
            self.fixed_sample_ratio, self.novelty_ratio = curriculum_ratios(epoch, max_epochs)
            print(f'  - Fixed sample ratio: {self.fixed_sample_ratio:.2f}')
            print(f'  - Novelty ratio: {self.novelty_ratio:.2f}')
            if epoch < max_epochs * 0.3:
                print('  - Using fixed sample strategy')
            self._refresh_training_samples()
        elif self.split == 'val':
            random.seed(42 + self.current_epoch)
            self.dynamic_fake = self._draw_dynamic()
            self.current_fake = self.core_fake + self.dynamic_fake

    def video_dir(self, index):
        """(frames directory, label) of item ``index``; counts a use of a train / val fake."""
        n_real = len(self.real_videos)
        if index < n_real:
            return self.real_videos[index], 0
        k = index - n_real
        fakes = self.current_fake if self.split in ('train', 'val') else self.fake_videos
        if k >= len(fakes):
            raise IndexError(f"Index '{index}' out of range")
        d = fakes[k]['path']
        if self.split in ('train', 'val'):
            self.video_usage_counts[d] = self.video_usage_counts.get(d, 0) + 1
        return d, 1

    def __getitem__(self, index):
        d, label = self.video_dir(index)
        return self._clip(d), label


# ------------------------------------------------------------------ Celeb-DF v2
def parse_celebdf_test_list(path):
    """{'real': ids, 'fake': ids} of a Celeb-DF testing list, YouTube rows skipped
    (data_loader.py:380-418)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f"Testing file '{path}' not found")
    ids, youtube = {'real': [], 'fake': []}, 0
    with open(path) as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith('//'):
                continue
            parts = line.split()
            if len(parts) < 2:
                continue
            label, vpath = parts[0], parts[1]
            low = vpath.lower()
            if 'youtube' in low:
                youtube += 1
                continue
            vid = vpath.split('/')[-1].split('.')[0]
            if label == '1' and 'celeb-real' in low:
                ids['real'].append(vid)
            elif label == '0' and 'celeb-synthesis' in low:
                ids['fake'].append(vid)
    print(f'Skipped {youtube} YouTube videos')
    return ids


class CelebDFLoader(_ClipDataset):
    """Celeb-DF v2 clips (reference config/data_loader.py:342-538).  ``split`` is a list; with
    'test' in it (the default ['train', 'test'] included) the listed test videos are used."""

    _jpg_fallback = False

    def __init__(self, root, split=['train', 'test'], frame_count=24, transform=None, testing_file=None):  # noqa: B006
        super().__init__()
        self.root, self.split, self.frame_count = root, split, frame_count
        self.transform, self.testing_file = transform, testing_file
        self.real_videos, self.synthetic_videos = self._load_frames_dirs()
        print(f'Loaded {len(self.real_videos)} real videos and {len(self.synthetic_videos)} synthetic videos')

    def __len__(self):
        return len(self.real_videos) + len(self.synthetic_videos)

    def _load_split(self):
        return parse_celebdf_test_list(self.testing_file)

    def _load_frames_dirs(self):
        real_dir = os.path.join(self.root, 'celebdf/frames/Celeb-real')
        synth_dir = os.path.join(self.root, 'celebdf/frames/Celeb-synthesis')
        if not os.path.exists(real_dir):
            raise FileNotFoundError(f"Real videos frames directory '{real_dir}' not found")
        if not os.path.exists(synth_dir):
            raise FileNotFoundError(f"Synthetic videos frames directory '{synth_dir}' not found")

        def videos(d):           # os.listdir order, as the reference
            return [(v, os.path.join(d, v)) for v in os.listdir(d) if os.path.isdir(os.path.join(d, v))]
        test = self._load_split() if self.testing_file else {'real': [], 'fake': []}
        testing = 'test' in self.split

        def keep(items, listed):
            out = []
            for vid, path in items:
                if (vid in listed) if testing else (vid not in listed and path not in out):
                    out.append(path)
            return out
        return keep(videos(real_dir), test['real']), keep(videos(synth_dir), test['fake'])

    def __getitem__(self, index):
        if index < len(self.real_videos):
            d, label = self.real_videos[index], 0
        else:
            k = index - len(self.real_videos)
            if k >= len(self.synthetic_videos):
                raise IndexError(f"Index '{index}' out of range")
            d, label = self.synthetic_videos[k], 1
        return self._clip(d), label


# ------------------------------------------------------------------ diffusion images
class DiffusionLoader(Dataset):
    """Single images of diffusion-generated and real faces as 1-frame clips (reference
    config/data_loader.py:540-711)."""

    imread = staticmethod(imread_rgb)

    def __init__(self, root, frame_count=1, transform=None, methods=['DDPM', 'DDIM', 'LDM'],  # noqa: B006
                 single_method=None):
        super().__init__()
        self.root, self.frame_count, self.transform = root, frame_count, transform
        self.single_method = single_method
        self.methods = [single_method] if single_method else methods
        self.real_images, self.fake_images = self._load_image_paths()
        print(f'Loaded {len(self.real_images)} real images and {len(self.fake_images)} fake images')
        counts = {}
        for v in self.fake_images:
            counts[v['method']] = counts.get(v['method'], 0) + 1
        print('Fake images by method:')
        for m, c in counts.items():
            print(f'  - {m}: {c} images')

    def __len__(self):
        return len(self.real_images) + len(self.fake_images)

    @staticmethod
    def _images(d):
        return [f for f in os.listdir(d) if f.endswith('.jpg') or f.endswith('.png')]

    def _load_image_paths(self):
        real, fake = [], []
        real_dir = os.path.join(self.root, 'CelebA-Real')
        if os.path.exists(real_dir):
            real = [os.path.join(real_dir, f) for f in self._images(real_dir)]
        else:
            print(f"Warning: Real images directory '{real_dir}' not found")
        for m in self.methods:
            mdir = os.path.join(self.root, m)
            if not os.path.exists(mdir):
                print(f"Warning: Method directory '{mdir}' not found")
                continue
            fake += [{'path': os.path.join(mdir, f), 'method': m, 'filename': f} for f in self._images(mdir)]
        real.sort()
        fake.sort(key=lambda v: v['path'])
        return real, fake

    def _entry(self, index):
        if index < len(self.real_images):
            p = self.real_images[index]
            return {'path': p, 'method': 'Real', 'label': 0, 'filename': os.path.basename(p)}
        k = index - len(self.real_images)
        if k >= len(self.fake_images):
            raise IndexError(f"Index '{index}' out of range")
        v = self.fake_images[k]
        return {'path': v['path'], 'method': v['method'], 'label': 1, 'filename': v['filename']}

    def __getitem__(self, index):
        e = self._entry(index)
        img = type(self).imread(e['path'])
        if img is None:
            raise FileNotFoundError(f"Could not load image from '{e['path']}'")
        if self.transform:
            img = self.transform.batch([img])[0] if hasattr(self.transform, 'batch') else self.transform(img)
        if not isinstance(img, torch.Tensor):
            raise TypeError(f'Transform should return torch.Tensor, got {type(img)}')
        return img.unsqueeze(0), e['label']

    def get_image_info(self, index):
        return self._entry(index)
