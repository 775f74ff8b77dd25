"""Probe: does the process group's flight-recorder dump show the watchdog's progress?

Eager RCCL collectives are queued to ProcessGroupNCCL's watchdog thread, which polls their
end events and retires them (pg_status last_completed_collective).  Prints the pg_status
right after a device synchronize and then every 20 ms until the watchdog has caught up.
"""
import json
import os
import socket
import time

import torch
import torch.distributed as dist
import torch._C._distributed_c10d as c10d


def status():
    d = json.loads(c10d._dump_nccl_trace_json(includeCollectives=True, onlyActive=False))
    return {'pg_status': d.get('pg_status', {}), 'entries': [(e.get('collective_seq_id'), e.get('state'), e.get('retired'))
                                                             for e in d.get('entries', [])][-3:]}


def main():
    os.environ.setdefault('TORCH_FR_BUFFER_SIZE', '2000')
    os.environ.setdefault('TORCH_NCCL_TRACE_BUFFER_SIZE', '2000')
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    x = torch.ones(1 << 20, device='cuda')
    print('before any collective:', status(), flush=True)
    for _ in range(5):
        dist.all_reduce(x)
    w = dist.all_reduce(x, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(40):
        st = status()
        print(f'{1e3 * (time.perf_counter() - t0):7.1f} ms', st, flush=True)
        ps = st['pg_status']
        if ps and all(v.get('last_completed_collective') == v.get('last_enqueued_collective') for v in ps.values()):
            break
        time.sleep(0.02)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
