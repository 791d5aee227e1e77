#!/usr/bin/env python3
"""Per-round timeline from a rocprofv3 kernel trace (tools/gpu.sh trace):
resolve duration, resolve-to-resolve gap, and the kernels around one resolve.

    python tools/trace_timeline.py gpurun_out/trace_<tag>/run_kernel_trace.csv [round]
"""
import csv
import statistics
import sys

KN = ['sweep_kernel', 'merge_shards', 'merge_kernel', 'resolve_kernel', 'patch_kernel', 'gather_cand', 'advance',
      'writeback', 'norm_check', 'streamOpsWait', 'streamOpsWrite']


def name(n):
    for k in KN:
        if k in n:
            return k
    return n[:24]


rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), name(r['Kernel_Name'])) for r in rows)
res = [e for e in ev if e[2] == 'resolve_kernel']
mid = res[len(res) // 4: 3 * len(res) // 4]
print(f"resolves {len(res)}  mean dur {statistics.mean((e[1] - e[0]) / 1e3 for e in mid):.1f} us  "
      f"mean start-to-start {statistics.mean((b[0] - a[0]) / 1e3 for a, b in zip(mid, mid[1:])):.1f} us  "
      f"mean end-to-start gap {statistics.mean((b[0] - a[1]) / 1e3 for a, b in zip(mid, mid[1:])):.1f} us")
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(res) // 2
t0 = res[k][0]
for s, e, n in ev:
    if res[k - 1][0] <= s <= res[k + 1][1]:
        print(f"{n:16s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  dur {(e - s) / 1e3:7.1f}")
