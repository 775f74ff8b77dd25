"""ORACLE (test infrastructure only) — numpy restatement of the Haar DWT and the
bilinear upsample the reference's MWT applies to it.

Reference call sites:
* ``network/mwt.py:20``  ``DWTForward(J=1, wave='haar', mode='zero')``
* ``network/mwt.py:76``  ``ll, hf = self.dwt(x)``
* ``network/mwt.py:77``  ``hf[0].reshape(B, 3*C, H//2, W//2)``  (channel = c*3 + band)
* ``network/mwt.py:79-81`` ``F.interpolate(hf, size=target_size, mode='bilinear')``
  (align_corners=False, no antialias) whenever ``levels > 1``.

Third-party algorithm restated: pytorch_wavelets (unpinned in
requirements.txt:9; latest 1.3.0) ``lowlevel.AFB2D`` for ``mode='zero'``:
a row pass (dim 3) then a column pass (dim 2), each a grouped stride-2
cross-correlation with the time-reversed pywt haar filters
``h0 = [s, s]``, ``h1 = [s, -s]``, ``s = float32(1/sqrt(2))``, giving per
channel the 4 outputs [LL, (W-lo,H-hi), (W-hi,H-lo), (W-hi,H-hi)];
``yh = y[:, :, 1:]`` is ``[B, C, 3, h, w]``.  Odd sizes are zero-padded by one
trailing sample (``pywt.dwt_coeff_len`` = ceil(N/2)).  Pinned against pywt
1.1.1 ``dwt2(x, 'haar', mode='zero')`` in tests/golden/dwt_pywt.npz.
"""
import numpy as np

S = np.float32(0.7071067811865476)  # float32(dec_lo[0]) — both filter taps


def _pad_even(x, axis):
    if x.shape[axis] % 2 == 0:
        return x
    pad = [(0, 0)] * x.ndim
    pad[axis] = (0, 1)
    return np.pad(x, pad)


def haar_level(x):
    """One analysis level.  x: float32 [B, C, H, W] -> (ll [B,C,h,w], yh [B,C,3,h,w]).

    Two fp32 passes exactly as AFB2D: row pass then column pass, each
    ``s*x[2n] + s*x[2n+1]`` / ``s*x[2n] - s*x[2n+1]``.
    """
    x = np.asarray(x, dtype=np.float32)
    x = _pad_even(_pad_even(x, 3), 2)
    e, o = x[..., 0::2], x[..., 1::2]
    lo_w = (S * e + S * o).astype(np.float32)
    hi_w = (S * e - S * o).astype(np.float32)

    def col(t):
        te, to = t[..., 0::2, :], t[..., 1::2, :]
        return (S * te + S * to).astype(np.float32), (S * te - S * to).astype(np.float32)

    ll, lh = col(lo_w)      # (W-lo,H-lo), (W-lo,H-hi)
    hl, hh = col(hi_w)      # (W-hi,H-lo), (W-hi,H-hi)
    yh = np.stack([lh, hl, hh], axis=2)
    return ll, yh


def haar_multilevel(x, levels):
    """Repeated J=1 DWT as MWT.forward's level loop does (mwt.py:107-111):
    returns (ll_last, [yh_level1, ..., yh_levelL])."""
    ll = np.asarray(x, dtype=np.float32)
    yhs = []
    for _ in range(levels):
        ll, yh = haar_level(ll)
        yhs.append(yh)
    return ll, yhs


def _src_index(out_size, in_size):
    """PyTorch area_pixel_compute_source_index, align_corners=False, linear."""
    scale = np.float32(in_size) / np.float32(out_size)
    d = np.arange(out_size, dtype=np.float32)
    src = scale * (d + np.float32(0.5)) - np.float32(0.5)
    src = np.maximum(src, np.float32(0.0)).astype(np.float32)
    i0 = np.floor(src).astype(np.int64)
    i0 = np.minimum(i0, in_size - 1)
    i1 = np.minimum(i0 + 1, in_size - 1)
    l1 = (src - i0.astype(np.float32)).astype(np.float32)
    l0 = (np.float32(1.0) - l1).astype(np.float32)
    return i0, i1, l0, l1


def bilinear(x, out_hw):
    """F.interpolate(x, size=out_hw, mode='bilinear', align_corners=False)."""
    x = np.asarray(x, dtype=np.float32)
    oh, ow = out_hw
    ih, iw = x.shape[-2:]
    if (oh, ow) == (ih, iw):
        return x.copy()
    h0, h1, hl0, hl1 = _src_index(oh, ih)
    w0, w1, wl0, wl1 = _src_index(ow, iw)
    top = x[..., h0, :]
    bot = x[..., h1, :]
    t = top[..., w0] * wl0 + top[..., w1] * wl1
    b = bot[..., w0] * wl0 + bot[..., w1] * wl1
    return (t * hl0[:, None] + b * hl1[:, None]).astype(np.float32)


def hf_upsampled(x, levels):
    """The MWT per-level high-frequency input of hf_conv (mwt.py:76-81):
    returns [levels, B, 3C, H//2, W//2] float32 (channel = c*3 + band)."""
    x = np.asarray(x, dtype=np.float32)
    B, C, H, W = x.shape
    target = (H // 2, W // 2)
    out = []
    ll = x
    for _ in range(levels):
        b, c, h, w = ll.shape
        ll_next, yh = haar_level(ll)
        hf = yh.reshape(b, 3 * c, yh.shape[-2], yh.shape[-1])
        if levels > 1:
            hf = bilinear(hf, target)
        out.append(hf)
        ll = ll_next
    return np.stack(out, 0)
