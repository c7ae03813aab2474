"""Per-lane walk statistics from ULG_WALK_CLOCK dumps: steps (loop
iterations the lane was active in), decision and open-node count."""
import glob, os, sys
import numpy as np
d = sys.argv[1]
for fn in sorted(glob.glob(os.path.join(d, "wclock_L*_p*.bin"))):
    a = np.fromfile(fn, dtype=np.uint64)
    qn = int(a[0])
    body = a[1:]
    # layout: 2 * (waves + 1) words, then one word per lane slot
    nslots = None
    for waves in range(1, len(body)):
        if 2 * (waves + 1) + waves * 64 == len(body):
            nslots = waves * 64
            off = 2 * (waves + 1)
            break
    if nslots is None or qn == 0:
        continue
    lanes = body[off:off + qn]
    steps = (lanes & np.uint64(0x7FFFFFFF)).astype(np.int64)
    dom = ((lanes >> np.uint64(31)) & np.uint64(1)).astype(bool)
    pc = (lanes >> np.uint64(32)).astype(np.int64)
    q = np.percentile(steps, [50, 90, 99, 99.9, 100])
    print(f"{os.path.basename(fn)}: lanes {qn}, dom {dom.mean():.2f}, steps p50/p90/p99/p99.9/max "
          f"{q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}/{q[3]:.0f}/{q[4]:.0f}, mean {steps.mean():.0f}; "
          f"corr(steps, open count) {np.corrcoef(steps, pc)[0, 1]:.2f}; "
          f"steps of top-1% by open count: {steps[pc >= np.percentile(pc, 99)].mean():.0f}")
