import sys, torch
sys.path[:0] = ['efficient-wavelet-vit_amd']
import ewvit
torch.manual_seed(3)
x = torch.randn(8, 3, 64, 64, device='cuda')
w = (torch.randn(24, 3, 3, 3, device='cuda') / 5).contiguous(memory_format=torch.channels_last)
ref = torch.nn.functional.conv2d(x.bfloat16().double(), w.bfloat16().double(), stride=2, padding=1)
y = ewvit.conv.stem_conv2d(x, w, None, 2).double()
with torch.autocast('cuda', dtype=torch.bfloat16):
    ym = torch.nn.functional.conv2d(x, w, stride=2, padding=1).double()
for name, t in (('ewvit', y), ('miopen', ym)):
    e = (t - ref).abs() / ref.abs().clamp_min(1e-3)
    print(name, 'max rel elem err', float(e.max()), 'mean', float(e.mean()), 'var', t.var(dim=(0,2,3))[:4].tolist())
print('ref var', ref.var(dim=(0,2,3))[:4].tolist())
