"""SURVEY §8 row N4, the data_loader.py half: config/data_loader.py (ours) against the
reference's own loaders, bit-exactly, on CPU.

tests/golden/ref_loader.json was written by tests/golden/gen_loader_golden.py, which ran the
reference's FaceForensicsLoader / CelebDFLoader / DiffusionLoader (config/data_loader.py) on the
synthetic tree of tests/loader_tree.py.  Here the same tree is rebuilt and our classes run the
same sequence: the same Python `random` seeds, construction, `update_sampling_strategy(epoch,
10)` for 10 epochs, `__getitem__` over every index (plus past-the-end) in the same order each
epoch.  Compared exactly: the real / fake video lists, `current_fake` after every epoch (the
curriculum of data_loader.py:171-269), the fixed / novelty ratios, the files each clip reads
(np.linspace selection, repeat-last padding: :305-320), the clip contents (blank frame for an
unreadable file: :325-331), labels, usage counts and the IndexError / FileNotFoundError cases.
"""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

import loader_tree


@pytest.fixture(scope='module')
def ref():
    with open(os.path.join(GOLDEN, 'ref_loader.json')) as f:
        return json.load(f)


@pytest.fixture(scope='module')
def tree(tmp_path_factory):
    return loader_tree.build(str(tmp_path_factory.mktemp('loader') / 'data'))


READS = []


def _logging(cls):
    from config import data_loader as D

    class Logged(cls):
        @staticmethod
        def imread(path):
            READS.append(path)
            return D.imread_rgb(path)
    return Logged


def _item(ds, root, i):
    READS.clear()
    try:
        clip, label = ds[i]
    except (IndexError, FileNotFoundError, TypeError, RuntimeError) as e:
        return {'index': i, 'error': type(e).__name__}
    return {'index': i, 'label': int(label), 'reads': [loader_tree.rel(root, p) for p in READS],
            'shape': list(clip.shape), 'clip_sha1': loader_tree.digest(clip)}


def _cases(ref, loader):
    return [c for c in ref['cases'] if c['loader'] == loader]


def test_fixture_covers_the_branches(ref):
    """the fixture exercises every branch it claims to"""
    ff = _cases(ref, 'FaceForensicsLoader')
    items = [it for c in ff for e in c['epochs'] for it in e['items']]
    assert any(it.get('error') == 'IndexError' for it in items)
    assert any(len(set(it.get('reads', []))) < len(it.get('reads', [])) for it in items)   # repeat-last padding
    assert any(any(r.endswith('.jpg') for r in it.get('reads', [])) for it in items)       # *.jpg fallback
    train = [c for c in ff if c['split'] == 'train' and not c['kw']]
    ratios = {tuple(e['ratios']) for c in train for e in c['epochs'] if e['epoch'] is not None}
    assert (1.0, 0.0) in ratios and (0.0, 1.0) in ratios and len(ratios) >= 4             # whole curriculum
    assert len({tuple(e['current_fake']) for c in train for e in c['epochs']}) > 10


@pytest.mark.parametrize('k', range(8))
def test_faceforensics_matches_reference(ref, tree, k):
    from config import data_loader as D
    case = _cases(ref, 'FaceForensicsLoader')[k]
    random.seed(case['seed'])
    ds = _logging(D.FaceForensicsLoader)(tree, split=case['split'], frame_count=case['frame_count'],
                                          transform=loader_tree.clip_transform, **case['kw'])
    assert [loader_tree.rel(tree, p) for p in ds.real_videos] == case['real']
    assert [{k2: (loader_tree.rel(tree, v[k2]) if k2 == 'path' else v[k2]) for k2 in ('path', 'method', 'target',
                                                                                       'source')}
            for v in ds.fake_videos] == case['fake']
    assert len(ds) == case['len']
    order = np.random.default_rng(case['seed'])
    epochs = iter(case['epochs'])
    for ep in [None] + (list(range(10)) if case['split'] in ('train', 'val') else []):
        want = next(epochs)
        if ep is not None:
            ds.update_sampling_strategy(ep, 10)
        assert want['epoch'] == ep and len(ds) == want['len']
        if case['split'] in ('train', 'val'):
            assert [loader_tree.rel(tree, v['path']) for v in ds.current_fake] == want['current_fake'], ep
        if case['split'] == 'train':
            assert [ds.fixed_sample_ratio, ds.novelty_ratio] == want['ratios']
        idx = order.permutation(len(ds) + 2).tolist()
        got = [_item(ds, tree, int(i)) for i in idx]
        assert got == want['items'], ep
        assert sorted([loader_tree.rel(tree, p), v] for p, v in ds.video_usage_counts.items()) == want['usage']


@pytest.mark.parametrize('k', range(2))
def test_celebdf_matches_reference(ref, tree, k):
    from config import data_loader as D
    case = _cases(ref, 'CelebDFLoader')[k]
    ds = _logging(D.CelebDFLoader)(tree, split=case['split'], frame_count=case['frame_count'],
                                    transform=loader_tree.clip_transform,
                                    testing_file=os.path.join(tree, 'celebdf', 'List_of_testing_videos.txt'))
    assert sorted(loader_tree.rel(tree, p) for p in ds.real_videos) == case['real']
    assert sorted(loader_tree.rel(tree, p) for p in ds.synthetic_videos) == case['fake']
    assert len(ds) == case['len']
    paths = list(ds.real_videos) + list(ds.synthetic_videos)
    got = {loader_tree.rel(tree, p): _item(ds, tree, i) for i, p in enumerate(paths)}
    # the reference walks os.listdir order, so item indices follow the directory order of the
    # tree it ran on: compare per video
    for key, want in case['items'].items():
        g = dict(got[key])
        w = dict(want)
        g.pop('index'), w.pop('index')
        assert g == w, key
    assert _item(ds, tree, len(ds))['error'] == case['past_end']['error']


@pytest.mark.parametrize('k', range(2))
def test_diffusion_matches_reference(ref, tree, k):
    from config import data_loader as D
    case = _cases(ref, 'DiffusionLoader')[k]
    droot = os.path.join(tree, 'diffusion')
    ds = _logging(D.DiffusionLoader)(droot, transform=loader_tree.clip_transform, single_method=case['single_method'])
    assert [loader_tree.rel(droot, p) for p in ds.real_images] == case['real']
    assert [{'path': loader_tree.rel(droot, v['path']), 'method': v['method'], 'filename': v['filename']}
            for v in ds.fake_images] == case['fake']
    assert [_item(ds, droot, i) for i in range(len(ds) + 1)] == case['items']
    assert [{kk: (loader_tree.rel(droot, v) if kk == 'path' else v) for kk, v in ds.get_image_info(i).items()}
            for i in range(len(ds))] == case['info']


def test_select_frames_rule():
    """np.linspace selection vs repeat-last padding (data_loader.py:311-320)"""
    from config import data_loader as D
    files = [f'{i}.png' for i in range(10)]
    assert D.select_frames(files, 4) == ['0.png', '3.png', '6.png', '9.png']
    assert D.select_frames(files[:3], 5) == ['0.png', '1.png', '2.png', '2.png', '2.png']
    assert D.select_frames(files, 10) == files
    with pytest.raises(IndexError):
        D.select_frames([], 2)


def test_curriculum_ratios():
    from config import data_loader as D
    assert D.curriculum_ratios(0, 10) == (1.0, 0.0)
    assert D.curriculum_ratios(2, 10) == (1.0, 0.0)
    f, n = D.curriculum_ratios(5, 10)
    assert f == pytest.approx(0.5) and n == pytest.approx(0.5)
    assert D.curriculum_ratios(9, 10) == (0.0, 1.0)
