"""Per-branch split of one training step from a rocprofv3 kernel trace of the EAGER bench
(`bench.py --eager`: the MWT runs on its own HIP stream, so the trace's Stream_Id separates
it; graph replay shows one queue).  Branches: MWT (side stream), backbone and token path
(main stream, told apart by kernel family), optimizer.  Step = the kernels between two
groups of Adam launches.  Usage: python tools/branch_split.py <run_kernel_trace.csv> [multi_adam_launches_per_step]"""
import collections
import csv
import re
import sys

TOKEN = re.compile(r'gemm_kernel|splitk_reduce|attn_|ln_fwd|ln_bwd|act_bwd|colsum|softmax|dropout|amax|'
                   r'log_sigmoid|sigmoid_kernel|neg_kernel|CatArray|at::native::reduce_kernel|combined_loss')
CONV_BB = re.compile(r'bn_|conv_|dw_|se_|stem_|scale_add|drop_add|pool')


def branch_of(name):
    if TOKEN.search(name) and not CONV_BB.search(name):
        return 'token path (ViT, cross-attention, heads, loss)'
    return 'backbone (EfficientNetV2-S) + glue'


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    adam = [i for i, r in enumerate(rows) if 'adam_table' in r['Kernel_Name']]
    aps = 1                                  # the single-launch Adam: one launch per step
    if not adam:                             # the per-48-tensor launches
        adam = [i for i, r in enumerate(rows) if 'adam_multi' in r['Kernel_Name']]
        aps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    ends = [adam[i] for i in range(aps - 1, len(adam), aps)]
    main_stream = collections.Counter(r['Stream_Id'] for r in rows).most_common(1)[0][0]
    # the last complete step that ran the MWT on its side stream (the bench's isolated
    # timing pass runs one stream)
    segs = [rows[a + 1:b + 1] for a, b in zip(ends, ends[1:])]
    seg = max(reversed(segs), key=lambda sg: sum(r['Stream_Id'] != main_stream for r in sg))
    agg = collections.defaultdict(lambda: [0, 0.0, None, None])
    for r in seg:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        n = r['Kernel_Name']
        if r['Stream_Id'] != main_stream:
            k = 'MWT (side stream)'
        elif 'adam_multi' in n:
            k = 'optimizer'
        else:
            k = branch_of(n)
        v = agg[k]
        v[0] += 1
        v[1] += (e - s) / 1e3
        v[2] = s if v[2] is None else min(v[2], s)
        v[3] = e if v[3] is None else max(v[3], e)
    t0 = min(int(r['Start_Timestamp']) for r in seg)
    t1 = max(int(r['End_Timestamp']) for r in seg)
    print(f'one eager step under rocprofv3: span {(t1 - t0) / 1e3:.1f} us (host-bound: eager launches under the '
          f'profiler), {len(seg)} kernels')
    print(f'{"branch":48s} {"kernels":>7s} {"kernel us":>10s} {"first..last (us from step start)":>34s}')
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f'{k:48s} {v[0]:7d} {v[1]:10.1f}   {(v[2] - t0) / 1e3:10.1f} .. {(v[3] - t0) / 1e3:10.1f}')


if __name__ == '__main__':
    main()
