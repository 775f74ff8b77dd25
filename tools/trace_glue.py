"""Per-step kernel table of one replayed step from a rocprofv3 --kernel-trace CSV (the window
between two consecutive Adam launches whose span is closest to the step time): the non-ewvit
(torch glue) kernels, and the total.  usage: python tools/trace_glue.py TRACE.csv STEP_MS"""
import collections
import csv
import sys


def main(path, step_ms):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    ad = [i for i, r in enumerate(rows) if 'adam_table' in r['Kernel_Name']]
    spans = [((int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e6, a, b) for a, b in zip(ad, ad[1:])]
    span, a, b = min(spans, key=lambda x: abs(x[0] - step_ms))
    win = rows[a + 1:b + 1]
    d = collections.defaultdict(list)
    for r in win:
        d[r['Kernel_Name'][:100]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    print(f'window {span:.2f} ms (profiled), {len(win)} kernels')
    tot = n = 0
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        if 'ewvit' in k:
            continue
        tot += sum(v)
        n += len(v)
        print(f'{sum(v):9.1f} us {len(v):5d}x  {k}')
    print(f'torch glue: {n} launches, {tot:.1f} us of kernel time')


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]))
