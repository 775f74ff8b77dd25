"""INTEGRATION.md §2 executed verbatim: the raw-ctypes reference-side
bindings a maintainer would paste — the DWT (replacing DWTForward at reference
network/mwt.py:20,76) and the frame loader (replacing the per-frame transform loop of
config/data_loader.py:325-337) — are read from INTEGRATION.md, run as written against
libewvit.so, and compared with the packaged path (ewvit.dwt_haar, FrameTransform.batch).
A snippet that drifts from include/ewvit.h fails here."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO

pytestmark = pytest.mark.gpu


def _section2_blocks():
    text = open(os.path.join(REPO, 'INTEGRATION.md')).read()
    sec = text[text.index('## 2.'):text.index('## 3.')]
    blocks = re.findall(r'```python\n(.*?)```', sec, re.S)
    assert len(blocks) == 2, 'INTEGRATION.md §2 should hold the DWT and the frames binding'
    return blocks


@pytest.fixture(scope='module')
def snippets():
    cwd = os.getcwd()
    os.chdir(REPO)                          # the snippets load the library by its repo-relative path
    try:
        ns = {}
        for b in _section2_blocks():
            exec(compile(b, 'INTEGRATION.md', 'exec'), ns)
    finally:
        os.chdir(cwd)
    return ns


def test_snippet_dwt_matches_package(snippets):
    import ewvit
    x = torch.randn(3, 3, 64, 48, device='cuda')
    ll, yh = snippets['dwt_haar'](x, levels=3)
    ll2, yh2 = ewvit.dwt_haar(x, 3)
    torch.cuda.synchronize()
    assert torch.equal(ll, ll2)
    assert len(yh) == len(yh2) == 3
    for a, b in zip(yh, yh2):
        assert a.shape == b.shape and torch.equal(a, b)


def test_snippet_frames_matches_package(snippets):
    from config.transforms import FrameTransform
    rng = np.random.default_rng(7)
    shapes = [(480, 640), (720, 1280), (300, 200)]
    frames = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]
    boxes = [(100, 40, 400, 380), (500, 100, 861, 470), (0, 50, 200, 250)]
    got = snippets['load_clip'](frames, boxes)
    ref = FrameTransform(device='cuda').batch(frames, boxes)
    torch.cuda.synchronize()
    assert got.shape == (3, 3, 224, 224)
    assert torch.equal(got, ref)
    with pytest.raises(ValueError):         # the plan's validation reaches the caller
        snippets['load_clip'](frames[:1], [(0, 0, 700, 700)])
