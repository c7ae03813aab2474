"""Per-wave wall-clock spans of the walk kernels (ULG_WALK_CLOCK=<dir>):
is a walk launch bound by total work or by its longest waves?"""
import glob, os, sys
import numpy as np
d = sys.argv[1]
for fn in sorted(glob.glob(os.path.join(d, "wclock_L*_p*.bin"))):
    a = np.fromfile(fn, dtype=np.uint64)
    qn = int(a[0])
    w = a[1:].reshape(-1, 2).astype(np.int64)
    w = w[w[:, 0] != 0]
    if len(w) == 0:
        continue
    t0 = w[:, 0].min()
    dur = (w[:, 1] - w[:, 0]) / 100.0  # wall_clock64 runs at 100 MHz -> us
    span = (w[:, 1].max() - t0) / 100.0
    starts = (w[:, 0] - t0) / 100.0
    q = np.percentile(dur, [50, 90, 99, 100])
    print(f"{os.path.basename(fn)}: queued {qn}, waves {len(w)}, kernel span {span:.1f} us, wave us p50/p90/p99/max "
          f"{q[0]:.1f}/{q[1]:.1f}/{q[2]:.1f}/{q[3]:.1f}, sum {dur.sum():.0f} us, last start {starts.max():.1f} us")
