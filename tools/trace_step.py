"""One training step from a rocprofv3 kernel trace: the kernels between the last two
launches of the DWT kernel (the first kernel of every forward), with durations, grid
and gaps.  Usage: python tools/trace_step.py <kernel_trace.csv> [--all] [--by-grid] [--nth K]"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [sys.argv[sys.argv.index('--marker') + 1]] if '--marker' in sys.argv else ['dwt_multilevel', 'dwt_hf_fused']
    starts = [i for i, r in enumerate(rows) if any(m in r['Kernel_Name'] for m in marks)]
    k = int(sys.argv[sys.argv.index('--nth') + 1]) if '--nth' in sys.argv else 2
    a, b = starts[-k], starts[-k + 1] if k > 1 else len(rows)
    if '--largest' in sys.argv:     # the delimited span with the most kernels (a whole step)
        spans = [(starts[i + 1] - starts[i], starts[i], starts[i + 1]) for i in range(len(starts) - 1)]
        _, a, b = max(spans)
    step = rows[a:b]
    t0 = int(step[0]['Start_Timestamp'])
    t1 = int(step[-1]['End_Timestamp'])
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in step)
    # busy = sum of kernel durations; union = time at least one kernel runs (overlap counted once)
    union, cur_s, cur_e = 0, None, None
    for r in sorted(step, key=lambda r: int(r['Start_Timestamp'])):
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += (cur_e - cur_s) if cur_e is not None else 0
    print(f'kernels {len(step)}  span {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  union {union / 1e6:.3f} ms '
          f'(idle {(t1 - t0 - union) / 1e6:.3f} ms)')
    agg = {}
    for r in step:
        n = r['Kernel_Name'].split('(')[0][:90]
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        c, t = agg.get(n, (0, 0))
        agg[n] = (c + 1, t + d)
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        print(f'{t / 1e3:9.1f} us {c:5d}  {n}')
    if '--by-grid' in sys.argv:
        # one row per (kernel, grid): the launch configurations of the step by total time
        agg = {}
        for r in step:
            n = r['Kernel_Name'].split('(')[0][:70]
            g = (r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'], r['Workgroup_Size_X'])
            d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            c, t = agg.get((n, g), (0, 0))
            agg[(n, g)] = (c + 1, t + d)
        print()
        for (n, g), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:120]:
            print(f'{t / 1e3:9.1f} us {c:4d}x {t / 1e3 / c:8.1f} us  {str(g):32s} {n}')
    if '--all' in sys.argv:
        prev = t0
        for r in step:
            s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            g = (r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
            print(f'{(s - t0) / 1e3:9.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:8.1f}  {g}  {r["Kernel_Name"][:100]}')
            prev = e


if __name__ == '__main__':
    main()
