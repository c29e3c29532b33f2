"""Reads the render service's per-claim take times (SPT_SVC_TRACE=1 +
SPT_SVC_TRACE_FILE, written by svc_end) and prints, per job, the percentiles of its
claims' take times and the blocks (and their XCD = block % 8) that took its last ones.
Usage: python tools/claim_trace.py FILE CLAIMS_PER_JOB"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
per = int(sys.argv[2])
t0, v = int(raw[0]), raw[1:]
taken = v != 0
t = ((v & np.uint64(0xFFFFFFFFFF)).astype(np.int64) - (t0 & 0xFFFFFFFFFF)) / 100.0  # us
blk = (v >> np.uint64(40)).astype(np.int64)
n = int(np.nonzero(taken)[0].max()) + 1
print(f"{n} claims taken, {per} per job")
for j in range(0, (n + per - 1) // per):
    sl = slice(j * per, min((j + 1) * per, n))
    tj, bj = t[sl][taken[sl]], blk[sl][taken[sl]]
    if not len(tj):
        continue
    p = np.percentile(tj, [0, 10, 50, 90, 99, 100])
    late = np.argsort(tj)[-8:]
    print(f"job {j}: take us p0 {p[0]:.0f} p10 {p[1]:.0f} p50 {p[2]:.0f} p90 {p[3]:.0f} p99 {p[4]:.0f} max {p[5]:.0f}; "
          f"last blocks {bj[late].tolist()} (xcd {(bj[late] % 8).tolist()}), their claims at job offset "
          f"{(np.arange(sl.start, sl.stop)[taken[sl]][late] - j * per).tolist()}")
