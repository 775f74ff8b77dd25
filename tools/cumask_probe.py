"""Probe: does a HIP stream's CU mask (hipExtStreamCreateWithCUMask) restrict the kernels
launched on it — eagerly, and when they were captured from it into a HIP graph?

A big memory-bound ewvit kernel (the MWT's BatchNorm apply over 2.4 M x 128 channels) is
timed on the default stream, on a stream masked to 1/4 of the CUs, and replayed from a graph
captured on the masked stream.  Masked should take ~4x as long if the mask is honoured.

  python tools/cumask_probe.py
"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'efficient-wavelet-vit_amd'))


def masked_stream(ncu, total):
    hip = ctypes.CDLL('libamdhip64.so')
    words = (total + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(ncu):
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f'hipExtStreamCreateWithCUMask rc={rc}')
    return torch.cuda.ExternalStream(s.value)


def main():
    import ewvit
    dev = torch.device('cuda', 0)
    total = torch.cuda.get_device_properties(dev).multi_processor_count
    x = torch.randn(192 * 112 * 112, 128, device=dev).to(torch.bfloat16)
    bn = torch.nn.BatchNorm1d(128).to(dev)

    def op():
        return ewvit.batch_norm_act(x, bn, 'relu', training=False)

    def timed(stream, fn, reps=20):
        with torch.cuda.stream(stream):
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                fn()
            e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / reps

    out = {'cus': total}
    out['default_us'] = timed(torch.cuda.current_stream(), op)
    ms = masked_stream(total // 4, total)
    out['masked_quarter_us'] = timed(ms, op)
    # captured on the masked stream, replayed on it and on the default stream
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(ms):
        op()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=ms):
            for _ in range(10):
                op()
    out['graph_replay_masked_stream_us'] = timed(ms, g.replay, 5) / 10
    out['graph_replay_default_stream_us'] = timed(torch.cuda.current_stream(), g.replay, 5) / 10
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == '__main__':
    main()
