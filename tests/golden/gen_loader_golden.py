"""Generate tests/golden/ref_loader.json: the reference's dataset classes
(/root/reference/config/data_loader.py — build container only; the reference never travels)
run on the synthetic tree of tests/loader_tree.py.

Recorded, per case (loader, split, Python `random` seed):
* the video lists the constructor builds (real / fake, with method, target, source);
* for FaceForensics train / val: `current_fake` after construction and after every
  `update_sampling_strategy(epoch, 10)` for epochs 0..9 (the curriculum of
  data_loader.py:171-269, driven by the global `random` state), plus the
  fixed / novelty ratios;
* `__getitem__` for every index in a seeded order each epoch (the usage counts that order
  the novelty pool depend on it): the label, the files cv2.imread was asked for (the
  np.linspace selection / repeat-last padding of :305-320) and the SHA-1 of the clip (the
  blank-frame branch of :325-331 for the unreadable file) through
  tests.loader_tree.clip_transform;
* the IndexError / FileNotFoundError cases.

cv2 is absent from the image: the stub reads images with Pillow and returns them in BGR
order (cv2.imread's IMREAD_COLOR: 8-bit, 3 channels) or None when the file cannot be
decoded, and cvtColor(BGR2RGB) reverses the channels — so the reference's own selection,
padding, blank-frame and stacking logic is what the fixture pins.

Usage:  python tests/golden/gen_loader_golden.py
"""
import json
import os
import random
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REF = '/root/reference'
sys.path.insert(0, TESTS)
sys.dont_write_bytecode = True

import loader_tree  # noqa: E402

READS = []


def install_cv2_stub():
    cv2 = types.ModuleType('cv2')
    cv2.COLOR_BGR2RGB = 4

    def imread(path):
        from PIL import Image
        READS.append(path)
        try:
            with Image.open(path) as im:
                rgb = np.asarray(im.convert('RGB'))
        except Exception:        # noqa: BLE001 — cv2.imread returns None for undecodable files
            return None
        return np.ascontiguousarray(rgb[..., ::-1])

    def cvtColor(img, code):
        assert code == cv2.COLOR_BGR2RGB
        return np.ascontiguousarray(img[..., ::-1])
    cv2.imread, cv2.cvtColor = imread, cvtColor
    sys.modules['cv2'] = cv2


def load_reference():
    install_cv2_stub()
    sys.path.insert(0, REF)
    import importlib.util
    spec = importlib.util.spec_from_file_location('ref_data_loader', os.path.join(REF, 'config', 'data_loader.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _video(root, v):
    return {k: (loader_tree.rel(root, v[k]) if k == 'path' else v[k]) for k in ('path', 'method', 'target', 'source')}


def _item(ds, root, i):
    READS.clear()
    try:
        clip, label = ds[i]
    except (IndexError, FileNotFoundError, TypeError, RuntimeError) as e:
        return {'index': i, 'error': type(e).__name__}
    return {'index': i, 'label': int(label), 'reads': [loader_tree.rel(root, p) for p in READS],
            'shape': list(clip.shape), 'clip_sha1': loader_tree.digest(clip)}


def ff_case(mod, root, split, seed, frame_count, epochs=10, **kw):
    random.seed(seed)
    ds = mod.FaceForensicsLoader(root, split=split, frame_count=frame_count, transform=loader_tree.clip_transform,
                                 **kw)
    case = {'loader': 'FaceForensicsLoader', 'split': split, 'seed': seed, 'frame_count': frame_count, 'kw': kw,
            'real': [loader_tree.rel(root, p) for p in ds.real_videos],
            'fake': [_video(root, v) for v in ds.fake_videos], 'len': len(ds), 'epochs': []}
    order = np.random.default_rng(seed)

    def snapshot(epoch):
        e = {'epoch': epoch, 'len': len(ds)}
        if split in ('train', 'val'):
            e['current_fake'] = [loader_tree.rel(root, v['path']) for v in ds.current_fake]
        if split == 'train':
            e['ratios'] = [ds.fixed_sample_ratio, ds.novelty_ratio]
        idx = order.permutation(len(ds) + 2).tolist()          # +2: past the end -> IndexError
        e['items'] = [_item(ds, root, int(i)) for i in idx]
        e['usage'] = sorted([loader_tree.rel(root, k), v] for k, v in ds.video_usage_counts.items())
        case['epochs'].append(e)
    snapshot(None)
    if split in ('train', 'val'):
        for ep in range(epochs):
            ds.update_sampling_strategy(ep, epochs)
            snapshot(ep)
    return case


def celeb_case(mod, root, split, frame_count):
    lst = os.path.join(root, 'celebdf', 'List_of_testing_videos.txt')
    ds = mod.CelebDFLoader(root, split=split, frame_count=frame_count, transform=loader_tree.clip_transform,
                           testing_file=lst)
    return {'loader': 'CelebDFLoader', 'split': split, 'frame_count': frame_count,
            'real': sorted(loader_tree.rel(root, p) for p in ds.real_videos),
            'fake': sorted(loader_tree.rel(root, p) for p in ds.synthetic_videos), 'len': len(ds),
            'items': {loader_tree.rel(root, p): _item(ds, root, i)
                      for i, p in enumerate(list(ds.real_videos) + list(ds.synthetic_videos))},
            'past_end': _item(ds, root, len(ds))}


def diffusion_case(mod, root, single_method=None):
    ds = mod.DiffusionLoader(os.path.join(root, 'diffusion'), transform=loader_tree.clip_transform,
                             single_method=single_method)
    droot = os.path.join(root, 'diffusion')
    return {'loader': 'DiffusionLoader', 'single_method': single_method,
            'real': [loader_tree.rel(droot, p) for p in ds.real_images],
            'fake': [{'path': loader_tree.rel(droot, v['path']), 'method': v['method'], 'filename': v['filename']}
                     for v in ds.fake_images],
            'items': [_item(ds, droot, i) for i in range(len(ds) + 1)],
            'info': [{k: (loader_tree.rel(droot, v) if k == 'path' else v) for k, v in ds.get_image_info(i).items()}
                     for i in range(len(ds))]}


def main():
    mod = load_reference()
    out = {'generator': 'tests/golden/gen_loader_golden.py', 'cases': []}
    with tempfile.TemporaryDirectory() as tmp:
        root = loader_tree.build(os.path.join(tmp, 'data'))
        for seed in (0, 1, 7):
            out['cases'].append(ff_case(mod, root, 'train', seed, 8))
        out['cases'].append(ff_case(mod, root, 'train', 3, 5, fixed_sample_ratio=1.0, novelty_ratio=0.0))
        out['cases'].append(ff_case(mod, root, 'val', 5, 8))
        out['cases'].append(ff_case(mod, root, 'val', 11, 6))
        out['cases'].append(ff_case(mod, root, 'test', 2, 8))
        out['cases'].append(ff_case(mod, root, 'test', 2, 8, single_method='FaceSwap'))
        out['cases'].append(celeb_case(mod, root, ['train', 'test'], 6))
        out['cases'].append(celeb_case(mod, root, ['train'], 6))
        out['cases'].append(diffusion_case(mod, root))
        out['cases'].append(diffusion_case(mod, root, 'DDIM'))
    path = os.path.join(HERE, 'ref_loader.json')
    with open(path, 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print(f'wrote {path}: {len(out["cases"])} cases, {os.path.getsize(path) / 1024:.0f} KB')


if __name__ == '__main__':
    main()
