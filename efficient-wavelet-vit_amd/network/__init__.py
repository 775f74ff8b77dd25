"""Drop-in replacements for the reference's network/{mwt,sfe,dama,model}.py.

Same class names, constructor signatures, attribute names and state-dict keys;
the hot path runs on the ewvit HIP kernels (../ewvit, C-ABI include/ewvit.h).
"""
import os

import yaml

_PKG_CONFIG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'config',
                           'architecture.yaml')


def load_config(path='config/architecture.yaml'):
    """The reference opens 'config/architecture.yaml' relative to the cwd
    (dama.py:94, model.py:31); do the same, else use the packaged copy."""
    p = path if os.path.exists(path) else _PKG_CONFIG
    with open(p, 'r') as f:
        return yaml.safe_load(f)
