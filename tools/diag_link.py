import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), 'efficient-wavelet-vit_amd'), os.path.join(os.getcwd(), 'tests')]
import torch
import test_gpu_bn_link as T

class MP:
    def setattr(self, o, n, v): setattr(o, n, v)
mp = MP()
g = torch.Generator().manual_seed(5)
N = 32
x0 = torch.randn(N, 160, 14, 14, generator=g).to('cuda', torch.bfloat16).contiguous(memory_format=torch.channels_last)
dyo = torch.randn(N, 256, 7, 7, generator=g).to('cuda', torch.bfloat16).contiguous(memory_format=torch.channels_last)
import ewvit.bn as ebn, network.efficientnet as en
for chain in ([(5, 7)], [(5, 7), (5, 8)], [(5, 7), (5, 8), (6, 0), (6, 1)]):
    mods = T._features(chain)
    xin = x0
    dyin = dyo if chain[-1][0] == 6 else torch.randn(N, 160, 14, 14, generator=g).to('cuda', torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = {}
    for dws, bl in ((False, False), (True, False), (False, True), (True, True)):
        orig = T._run.__code__
        ebn._BWD_LINK = bl
        en._DW_STATS = dws
        # _run sets both from `linked`; replicate without it
        m = mods().to('cuda').to(memory_format=torch.channels_last).train()
        for mod in m.modules():
            if hasattr(mod, 'sd_prob'):
                mod.sd_prob = 0.0
        x = xin.clone().requires_grad_(True)
        with torch.autocast('cuda', dtype=torch.bfloat16):
            y = m(x)
        y.backward(dyin)
        torch.cuda.synchronize()
        res[(dws, bl)] = (y.detach().float(), x.grad.float())
    b = res[(False, False)]
    for k, v in res.items():
        print(chain, k, 'y cos %.8f eq %s' % (T._cos(b[0], v[0]), torch.equal(b[0], v[0])), 'gx cos %.8f' % T._cos(b[1], v[1]))
    # run-to-run determinism
