"""Generate tests/golden/dwt_pywt.npz — the independent pin of the Haar DWT.

pytorch_wavelets (the reference's DWT, mwt.py:5,20) is absent from the image;
its filter bank is pywt's.  pywt 1.1.1 is importable only from the image's
/opt/conda python3.9, so this script runs there:

    /opt/conda/bin/python3.9 tests/golden/gen_pywt_golden.py

pywt.dwt2(x, 'haar', mode='zero') returns (cA, (cH, cV, cD)); pytorch_wavelets'
yh[0][:, :, b] corresponds to (cH, cV, cD)[b].  Levels are
chained on cA as MWT.forward chains on ll (mwt.py:107-111).  Inputs are float32
(the reference's dtype); pywt computes in float32 for float32 input.
"""
import os

import numpy as np
import pywt

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rng = np.random.default_rng(42)
    out = {}
    cases = {'a': (2, 3, 16, 16), 'b': (1, 2, 24, 40), 'odd': (1, 1, 13, 10)}
    for name, shape in cases.items():
        x = rng.standard_normal(shape).astype(np.float32)
        out[f'{name}.x'] = x
        ll = x
        levels = 3 if name != 'odd' else 2
        for lv in range(1, levels + 1):
            cA, (cH, cV, cD) = pywt.dwt2(ll, 'haar', mode='zero', axes=(-2, -1))
            out[f'{name}.L{lv}.ll'] = cA.astype(np.float32)
            out[f'{name}.L{lv}.yh'] = np.stack([cH, cV, cD], axis=2).astype(np.float32)
            ll = cA.astype(np.float32)
    out['pywt_version'] = np.array(pywt.__version__)
    np.savez_compressed(os.path.join(HERE, 'dwt_pywt.npz'), **out)
    print('pywt', pywt.__version__, 'wrote', len(out), 'arrays')


if __name__ == '__main__':
    main()
