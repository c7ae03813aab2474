"""Distinct presence patterns among the lanes that run the dominance walk
(dumped by score_variant 13 with ULG_DUMP_DIR): the walk's visited set is a
function of (presence bits, whether variable 0 is in P) alone."""
import glob, os, sys
import numpy as np
d = sys.argv[1]
for fn in sorted(glob.glob(os.path.join(d, "walk_L*_p*.bin"))):
    L = int(os.path.basename(fn).split("_")[1][1:])
    W = 1 if L + 1 <= 6 else 1 << (L + 1 - 6)
    a = np.fromfile(fn, dtype=np.uint64).reshape(-1, 2 * W + 1)
    if len(a) == 0:
        continue
    pres = a[:, :W]
    flag = a[:, 2 * W] & np.uint64(3)
    steps = (a[:, 2 * W] >> np.uint64(8)).astype(np.int64)
    key = np.concatenate([pres, (flag >> np.uint64(1))[:, None]], axis=1)
    u, inv, cnt = np.unique(key, axis=0, return_inverse=True, return_counts=True)
    top = np.sort(cnt)[::-1]
    print(f"{os.path.basename(fn)}: walkers {len(a)}, distinct (presence, v0inP) {len(u)}, "
          f"top10 share {top[:10].sum() / len(a):.3f}, top1000 share {top[:1000].sum() / len(a):.3f}, "
          f"mean steps {steps.mean():.1f}")
