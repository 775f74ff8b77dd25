"""Layer-by-layer parity of the backbone in TRAIN mode: every EfficientNetV2-S block of the
product (network/efficientnet.py on the ewvit kernels, bf16 autocast) against the same block of
the fp32 CPU oracle (oracle/effnetv2.py, the torchvision V2-S restatement the reference calls at
network/sfe.py:150), both fed the SAME input — the oracle's own activation at that depth — so
no error accumulates from the layers before it.

The whole-step test (test_gpu_modules.py::test_dama_train_step_vs_oracle) has to allow the
spread of bf16 arithmetic through ~300 layers; here each block is held to the module bounds of
SURVEY §8c tightened to what the blocks measure (profiles/r03/layerwise_parity.jsonl: output
max |err| <= 0.78 % of scale and cosine >= 0.99998; weight-gradient cosines >= 0.99974; input-
gradient cosines >= 0.99998): output max |err| <= 1.5e-2 of scale, cosine >= 0.9999; every weight
gradient cosine >= 0.999 and its norm within 1 % of the oracle's (cosine is blind to a scale
error); input gradient cosine >= 0.9999 and norm within 1 % — so a systematic error of a
percent or more in any one deep layer fails its own block.  Train-mode BatchNorm over 8
frames (the reference's chunk statistics), stochastic depth off.  Biases before a train-mode BatchNorm have an exactly zero true gradient
(their computed gradient is rounding noise) and are left out.
"""
import pytest
import torch

from test_gpu_modules import DEV, check, cos, log, pair

pytestmark = pytest.mark.gpu


def _norm_ratio(a, b):
    return float(a.detach().double().cpu().norm() / max(float(b.detach().double().cpu().norm()), 1e-30))


@pytest.fixture(scope='module')
def backbone_pair():
    from network import dama
    from oracle import model as om
    torch.manual_seed(0)
    p, o = pair(dama.DAMA, om.DAMA, (3, 128, 4, 3, 8), 14)
    return p.sfe.efficient_net.features, o.sfe.efficient_net.features


def _blocks(feats):
    out = []
    for i, stage in enumerate(feats):
        if isinstance(stage, torch.nn.Sequential) and i not in (0, len(feats) - 1):
            out += [(f'{i}.{j}', (i, j)) for j in range(len(stage))]
        else:
            out.append((f'{i}', (i, None)))
    return out


def test_backbone_blocks_train_layerwise(backbone_pair):
    pf, of = backbone_pair
    pf.train()
    of.train()
    from oracle.weights import recipe_input
    g = torch.Generator().manual_seed(7)
    x = recipe_input((8, 3, 224, 224), seed=2024)
    worst = (1.0, None)
    checked = 0
    for name, (i, j) in _blocks(of):
        om = of[i] if j is None else of[i][j]
        pm = pf[i] if j is None else pf[i][j]
        xin = x.detach()
        trainable = [n for n, q in om.named_parameters() if q.requires_grad]
        # the oracle's activation at this depth, fed to both
        xo = xin.clone().requires_grad_(bool(trainable) and i > 0)
        yo = om(xo)
        dy = torch.randn(yo.shape, generator=g)
        xp = xin.to(DEV).to(memory_format=torch.channels_last).requires_grad_(xo.requires_grad)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            yp = pm(xp)
        check(yp, yo, 1.5e-2, 0.9999)
        if trainable:
            (yo * dy).sum().backward()
            (yp.float() * dy.to(DEV)).sum().backward()
            pp, oo = dict(pm.named_parameters()), dict(om.named_parameters())
            for n in trainable:
                if n.endswith('.bias') or oo[n].grad is None:
                    continue
                assert pp[n].grad is not None, f'{name}.{n}'
                c = cos(pp[n].grad, oo[n].grad)
                r = _norm_ratio(pp[n].grad, oo[n].grad)
                log(f'grad_cos:{name}.{n}', c, 0.999)
                log(f'grad_norm_ratio:{name}.{n}', r, 0.01)
                worst = min(worst, (c, f'{name}.{n}'))
                assert c >= 0.999, f'block {name} {n}: grad cosine {c:.5f}'
                assert abs(r - 1) <= 0.01, f'block {name} {n}: grad norm ratio {r:.5f}'
            if xo.requires_grad:
                c = cos(xp.grad, xo.grad)
                r = _norm_ratio(xp.grad, xo.grad)
                log(f'dx_cos:{name}', c, 0.9999)
                log(f'dx_norm_ratio:{name}', r, 0.01)
                assert c >= 0.9999, f'block {name}: input-gradient cosine {c:.5f}'
                assert abs(r - 1) <= 0.01, f'block {name}: input-gradient norm ratio {r:.5f}'
            for q in list(om.parameters()) + list(pm.parameters()):
                q.grad = None
            checked += 1
        x = yo.detach()
    log('grad_cos_worst:' + str(worst[1]), worst[0], 0.999)
    assert checked >= 35, checked


def _check_grads(name, pm, om, xp, xo, dx_cos=0.9999, w_cos=0.999):
    pp, oo = dict(pm.named_parameters()), dict(om.named_parameters())
    for n, q in oo.items():
        if not q.requires_grad or n.endswith('.bias') or q.grad is None:
            continue
        assert pp[n].grad is not None, f'{name}.{n}'
        c, r = cos(pp[n].grad, q.grad), _norm_ratio(pp[n].grad, q.grad)
        log(f'grad_cos:{name}.{n}', c, w_cos)
        log(f'grad_norm_ratio:{name}.{n}', r, 0.01)
        assert c >= w_cos and abs(r - 1) <= 0.01, f'{name} {n}: grad cosine {c:.5f}, norm ratio {r:.5f}'
    c, r = cos(xp, xo), _norm_ratio(xp, xo)
    log(f'dx_cos:{name}', c, dx_cos)
    log(f'dx_norm_ratio:{name}', r, 0.01)
    assert c >= dx_cos and abs(r - 1) <= 0.01, f'{name}: input-gradient cosine {c:.5f}, norm ratio {r:.5f}'


def test_mwt_modules_train_layerwise():
    """The MWT's conv-BN-ReLU stages alone in train mode (8 frames, the same non-negative input
    to both): hf_conv fusion (54 -> 128; the product reads the input zero-padded to 64 channels,
    as the step lays it out), multiscale_fusion over the three level-major maps (the product
    reads cat(x.chunk(3), 1) in place), freq_conv (stride 2) and freq_pool.  The seperate convs
    run as the grouped hfsep kernel inside the step (tests/test_gpu_hfsep.py).  Input gradients
    >= 0.999 here (not 0.9999): behind a ReLU the product's mask comes from the bf16-rounded
    pre-activation, and the elements that round across zero take or drop their gradient (the
    SiLU blocks above are smooth there).  freq_pool's conv weight gradient >= 0.997 and input
    gradient >= 0.998 (measured 0.9984 / 0.9988; the max-pool routes ties to the first maximum
    as torch does): its output gradient is one value per (frame, channel) spread by the average
    pool, so the BatchNorm backward's mean-removal cancels most of it and leaves the rounding."""
    from network import mwt as pmwt
    from oracle import model as om_
    from oracle.weights import recipe_state_dict
    torch.manual_seed(0)
    o = om_.MWT(3, 128, 3)
    sd = recipe_state_dict(o.state_dict(), 21)
    o.load_state_dict(sd)
    p = pmwt.MWT(3, 128, 3)
    p.load_state_dict(sd)
    p = p.to(DEV).train()
    o.train()
    g = torch.Generator().manual_seed(11)
    N, H = 8, 56
    cases = [
        ('hf_conv.fusion', p.hf_conv['fusion'], o.hf_conv['fusion'], (N, 54, H, H), 64, 1),
        ('multiscale_fusion', p.multiscale_fusion, o.multiscale_fusion, (3 * N, 128, H, H), 128, 3),
        ('freq_conv', p.freq_conv, o.freq_conv, (N, 128, H, H), 128, 1),
        ('freq_pool', p.freq_pool, o.freq_pool, (N, 128, H // 2, H // 2), 128, 1),
    ]
    for name, pm, om, shape, cpad, levels in cases:
        x = torch.relu(torch.randn(shape, generator=g)).to(torch.bfloat16).float()
        xo = x.clone().requires_grad_(True)
        yo = om(torch.cat(xo.chunk(levels), 1) if levels > 1 else xo)
        dy = torch.randn(yo.shape, generator=g)
        xpad = torch.zeros(shape[0], cpad, shape[2], shape[3])
        xpad[:, :shape[1]] = x
        xp = xpad.to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_(True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            yp = pm(xp, levels) if levels > 1 else pm(xp)
        check(yp, yo, 1.5e-2, 0.9999)
        (yo * dy).sum().backward()
        (yp.float() * dy.to(DEV)).sum().backward()
        _check_grads(name, pm, om, xp.grad[:, :shape[1]], xo.grad, dx_cos=0.998 if name == 'freq_pool' else 0.999,
                     w_cos=0.997 if name == 'freq_pool' else 0.999)
