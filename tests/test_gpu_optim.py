"""Multi-tensor Adam (csrc/optim.hip, ewvit.optim.Adam) vs torch.optim.Adam on the same
parameters and gradients (the reference's optimizer, train.py:273-275).

Tolerance: the kernel follows torch's foreach operation order with the bias corrections
in double; the compiler may still contract multiply-adds, so parameters and moments are
held to 1e-6 relative after several steps.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(7,), (64, 3, 3, 3), (128, 54, 3, 3), (1000, 13), (1536, 256, 1, 1), (5,)] + [(33, 17)] * 50
    ps = []
    for i, s in enumerate(shapes):
        t = torch.randn(s, generator=g)
        if len(s) == 4:
            t = t.to(memory_format=torch.channels_last)
        ps.append(t)
    return ps


@pytest.mark.parametrize('wd', [0.0, 1e-4])
def test_adam_matches_torch(wd):
    import ewvit
    base = _params(3)
    pt = [t.clone().to(DEV).requires_grad_(True) for t in base]
    pe = [t.clone().to(DEV).requires_grad_(True) for t in base]
    for a, b in zip(pt, pe):
        assert a.stride() == b.stride()
    ot = torch.optim.Adam(pt, lr=1e-3, weight_decay=wd)
    oe = ewvit.optim.Adam(pe, lr=1e-3, weight_decay=wd)
    g = torch.Generator().manual_seed(4)
    for step in range(4):
        for a, b in zip(pt, pe):
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad = gr.clone().to(memory_format=torch.channels_last) if a.dim() == 4 else gr.clone()
            b.grad = gr.clone().to(memory_format=torch.channels_last) if b.dim() == 4 else gr.clone()
        if step == 2:
            pe[0].grad = None       # a parameter without a gradient this step is skipped
            pt[0].grad = None
        ot.step()
        oe.step()
    for a, b in zip(pt, pe):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), float((a - b).abs().max())
        sa, sb = ot.state[a], oe.state[b]
        # exp_avg ~ |g| ~ 1 crosses zero (lerp cancels): absolute floor of a few f32 ulps at 1
        assert torch.allclose(sa['exp_avg'], sb['exp_avg'], rtol=1e-6, atol=1e-7), \
            float((sa['exp_avg'] - sb['exp_avg']).abs().max())
        assert torch.allclose(sa['exp_avg_sq'], sb['exp_avg_sq'], rtol=1e-6, atol=1e-10), \
            float((sa['exp_avg_sq'] - sb['exp_avg_sq']).abs().max())
    assert float(oe.state[pe[1]]['step']) == 4.0


def test_adam_state_dict_roundtrip():
    """torch.optim.Adam state (per-parameter step / exp_avg / exp_avg_sq) loads into
    ewvit.optim.Adam and training continues identically."""
    import ewvit
    base = _params(5)[:6]
    pt = [t.clone().to(DEV).requires_grad_(True) for t in base]
    pe = [t.clone().to(DEV).requires_grad_(True) for t in base]
    ot = torch.optim.Adam(pt, lr=2e-3, weight_decay=1e-4)
    g = torch.Generator().manual_seed(6)
    grads = [[torch.randn(p.shape, generator=g).to(DEV) for p in pt] for _ in range(3)]
    for k in range(2):
        for p, gr in zip(pt, grads[k]):
            p.grad = gr.clone()
        ot.step()
    with torch.no_grad():
        for a, b in zip(pe, pt):
            a.copy_(b)
    oe = ewvit.optim.Adam(pe, lr=2e-3, weight_decay=1e-4)
    oe.load_state_dict(copy.deepcopy(ot.state_dict()))   # load_state_dict aliases same-device tensors
    for p, q, gr in zip(pt, pe, grads[2]):
        p.grad = gr.clone()
        q.grad = gr.clone()
    ot.step()
    oe.step()
    for a, b in zip(pt, pe):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)


def test_adam_table_launch_matches_per_tensor_launches():
    """the one-launch form (device table) against the 48-tensors-per-launch form, bit-exact,
    and against torch; the table is rebuilt when a gradient moves"""
    import ewvit
    base = _params(5)
    pa = [t.clone().to(DEV).requires_grad_(True) for t in base]
    pb = [t.clone().to(DEV).requires_grad_(True) for t in base]
    oa = ewvit.optim.Adam(pa, lr=1e-3, weight_decay=1e-4)
    ob = ewvit.optim.Adam(pb, lr=1e-3, weight_decay=1e-4)
    oa.table, ob.table = True, False
    g = torch.Generator().manual_seed(6)
    tab_ptrs = []
    for step in range(3):
        for a, b in zip(pa, pb):
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad = gr.clone().contiguous(memory_format=torch.channels_last) if a.dim() == 4 else gr.clone()
            b.grad = gr.clone().contiguous(memory_format=torch.channels_last) if b.dim() == 4 else gr.clone()
        oa.step()
        ob.step()
        tab_ptrs.append(oa._tables[0][1].data_ptr())
    torch.cuda.synchronize()
    assert len(oa._tables) == 1 and not getattr(oa, '_table_keep', [])   # eager tables are not kept
    # new gradient addresses every step: the one device table is refilled in place (pinned
    # host staging), not reallocated
    assert len(set(tab_ptrs)) == 1
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
        assert torch.equal(oa.state[a]['exp_avg'], ob.state[b]['exp_avg'])
        assert torch.equal(oa.state[a]['exp_avg_sq'], ob.state[b]['exp_avg_sq'])
