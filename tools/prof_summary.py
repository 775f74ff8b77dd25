"""Per-category GPU time per step from a rocprofv3 --stats kernel_stats.csv.
Usage: python tools/prof_summary.py <kernel_stats.csv> <dispatch rounds (warmup+steps+timing)> [top]"""
import collections
import csv
import sys


def category(n):
    if 'bn_' in n:
        return 'ewvit BN'
    if 'conv_fwd' in n or 'conv_wgrad' in n or 'conv_pack' in n or 'conv3x3' in n:
        return 'ewvit conv'
    if n.startswith('igemm') or 'SubTensor' in n or 'ck::' in n or 'naive_conv' in n or 'batched_transpose' in n \
            or '_ZN2ck' in n:
        return 'MIOpen/CK conv'
    if 'dw_' in n:
        return 'ewvit depthwise'
    if 'gemm' in n or 'splitk' in n:
        return 'ewvit gemm'
    if 'attn' in n:
        return 'ewvit attention'
    if 'ln_' in n or 'layernorm' in n:
        return 'ewvit layernorm'
    if 'dwt' in n or 'hf_upsample' in n:
        return 'ewvit dwt'
    if 'copyBuffer' in n or 'copy' in n or 'CatArray' in n:
        return 'copies/cat'
    if 'reduce_kernel' in n:
        return 'torch reduce'
    if 'elementwise' in n:
        return 'torch elementwise'
    if 'multi_tensor' in n:
        return 'adam'
    return 'other'


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rounds = float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    cat = collections.defaultdict(float)
    for r in rows:
        cat[category(r['Name'])] += float(r['TotalDurationNs']) / rounds / 1e3
    print(f'total {sum(cat.values()):.1f} us/step')
    for k, v in sorted(cat.items(), key=lambda kv: -kv[1]):
        print(f'{v:9.1f} us  {k}')
    print()
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / rounds / 1e3:9.1f} us {int(r['Calls']) / rounds:6.1f}x "
              f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")


if __name__ == '__main__':
    main()
