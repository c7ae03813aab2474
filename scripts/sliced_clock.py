"""Per-wave spans and union points of the bit-sliced walk (ULG_WALK_CLOCK)."""
import glob, os, sys
import numpy as np
for fn in sorted(glob.glob(os.path.join(sys.argv[1], "sliced_L*_p*.bin"))):
    a = np.fromfile(fn, dtype=np.uint64).reshape(-1, 3).astype(np.int64)
    a = a[a[:, 0] != 0]
    if len(a) == 0:
        continue
    dur = (a[:, 1] - a[:, 0]) / 100.0
    span = (a[:, 1].max() - a[:, 0].min()) / 100.0
    pts = a[:, 2]
    print(f"{os.path.basename(fn)}: waves {len(a)}, span {span:.1f} us, wave us p50/p90/max "
          f"{np.percentile(dur, 50):.1f}/{np.percentile(dur, 90):.1f}/{dur.max():.1f}, points p50/p90/max "
          f"{np.percentile(pts, 50):.0f}/{np.percentile(pts, 90):.0f}/{pts.max()}, ns per point (median wave) "
          f"{np.median(dur * 1e3 / np.maximum(pts, 1)):.1f}")
