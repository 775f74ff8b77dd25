"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are KiB;
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores.

usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> [regex]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get('Counter_Name') != counter:
            continue
        per[r['Kernel_Name']].append(float(r['Counter_Value']))
    return per


def main():
    args = sys.argv[1:]
    steps = None
    if '--steps' in args:
        i = args.index('--steps')
        steps = int(args[i + 1])
        del args[i:i + 2]
    config = 2
    if '--config' in args:
        i = args.index('--config')
        config = int(args[i + 1])
        del args[i:i + 2]
    fetch = load(args[0], 'FETCH_SIZE')
    write = load(args[1], 'WRITE_SIZE')
    pat = re.compile(args[2]) if len(args) > 2 else None
    out = {'_steps_executed': steps, '_config': config,
           '_source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate); FETCH_SIZE x2 (gfx950 correction)'}
    for k in sorted(set(fetch) | set(write)):
        if pat and not pat.search(k):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        out[k[:160]] = {'dispatches': max(len(f), len(w)), 'fetch_bytes_x2': fb, 'write_bytes': wb,
                        'hbm_bytes_per_launch': (fb or 0) + (wb or 0)}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
